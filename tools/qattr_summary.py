"""Summarise a tools/gpu_qattr.sh run: per SME_QEXP part switch the k_query_win time
(tools/qexp.py) and the raw FETCH_SIZE of one batch, and the differences between
consecutive switches = the time / beyond-L2 bytes of each part of the kernel.

    python tools/qattr_summary.py [gpurun_out/qattr] [--pairs N] > profiles/<name>.json
"""
import csv
import glob
import json
import os
import sys

PARTS = [(0, "full kernel"), (2, "- exact candidate scoring"), (3, "- passing sub-block sums"),
         (7, "- sparse postings"), (15, "- heavy sub-block bounds (records / skip entries / pipeline left)")]
WHAT = {0: "candidates: tf bytes, LDS / global tf search, list appends",
        2: "passing sub-blocks: listing + exact A(d) from one heavy impact dword per term (+ sparse entries)",
        3: "sparse postings of the window: posting words, LDS block sums and list",
        7: "heavy sub-block bounds: sbq rows (one uint4 per heavy term and lane)",
        15: "per-pair overhead: position / term records, thresholds, skip entries"}


def counters(d):
    """{counter: total over the run's k_query_win dispatches} (FETCH_SIZE in bytes), dispatches"""
    tot, disp = {}, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_query_win" in r["Kernel_Name"]:
                v = float(r["Counter_Value"]) * (1024 if r["Counter_Name"] == "FETCH_SIZE" else 1)
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + v
                disp.add(r["Dispatch_Id"])
    return tot, len(disp)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    root = args[0] if args else "gpurun_out/qattr"
    pairs = None
    if "--pairs" in sys.argv:
        pairs = float(sys.argv[sys.argv.index("--pairs") + 1])
    rows = []
    for e, name in PARTS:
        t = None
        log = os.path.join(root, "time_%d.log" % e)
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{") and '"opts"' in line:
                    t = json.loads(line)
        cs, nd = counters(os.path.join(root, "f_%d" % e))
        row = {"qexp": e, "switch": name, "kernel_ms": t["kernel_ms"] if t else None,
               "fetch_bytes_raw_per_batch": round(cs.get("FETCH_SIZE", 0.0)), "dispatches": nd}
        for c, v in sorted(cs.items()):
            if c != "FETCH_SIZE":
                row[c] = round(v)
        rows.append(row)
    parts = []
    for a, b in zip(rows, rows[1:] + [None]):
        ms = a["kernel_ms"] - (b["kernel_ms"] if b else 0.0) if a["kernel_ms"] is not None else None
        fb = a["fetch_bytes_raw_per_batch"] - (b["fetch_bytes_raw_per_batch"] if b else 0)
        p = {"part": WHAT[a["qexp"]], "ms": round(ms, 3) if ms is not None else None, "fetch_bytes_raw": fb}
        if pairs:
            p["fetch_bytes_raw_per_pair"] = round(fb / pairs, 1)
        for c in [c for c in a if c.startswith("SQ_")]:
            p[c] = a[c] - (b.get(c, 0) if b else 0)
            if pairs:
                p[c + "_per_pair"] = round(p[c] / pairs, 1)
        parts.append(p)
    print(json.dumps({"runs": rows, "parts": parts, "pairs": pairs,
                      "method": "SME_QEXP part switches of the experiment build (timing only; results wrong by "
                                "design), each run timed by tools/qexp.py and measured by its own rocprofv3 --pmc "
                                "FETCH_SIZE pass; a part = the difference between consecutive switches"}, indent=1))


if __name__ == "__main__":
    main()
