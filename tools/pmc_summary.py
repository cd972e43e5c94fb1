"""Per-launch HBM traffic from rocprofv3 PMC passes -> profiles/pmc_traffic.json.

usage: python tools/pmc_summary.py DOCS VOCAB FETCH_DIR WRITE_DIR [KERNEL ...]

FETCH_DIR / WRITE_DIR hold the run_counter_collection.csv of two separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs of
`bench.py --docs DOCS --vocab VOCAB ...` (one counter group per run: FETCH_SIZE
takes 3 TCC slots, WRITE_SIZE 2).  Both counters are in KiB.  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE reports half the bytes of wide
streaming reads on gfx950, so the fetch side is doubled; WRITE_SIZE is exact
for 16-byte streaming stores.  Values are averaged over the kernel's dispatches
(warm-up builds included: a build's kernels see the same bytes every step).
"""
import csv
import glob
import json
import os
import sys


def base_name(n):
    """Kernel name without return type, template arguments or parameter list:
    'void k_query_win<true>(Args)' -> 'k_query_win'.  Kernels are matched on this
    EXACTLY (k_query must not collect k_query_win / k_query_seed / ...)."""
    n = n.strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    for c in "(<":
        i = n.find(c)
        if i >= 0:
            n = n[:i]
    # namespace qualifiers ('sme::k_tok_fast' -> 'k_tok_fast')
    return n.strip().rsplit("::", 1)[-1]


def per_kernel(d, counter):
    """{kernel name: [value per dispatch]} in dispatch order.  SME_PMC_BATCHES=n keeps
    only the dispatches before the (n+1)-th k_query_seed (the bench's headline query
    batches: warm-up + timed; the uniform-vocabulary batches follow them)."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    nb = int(os.environ.get("SME_PMC_BATCHES", "0"))
    out, seeds = {}, 0
    for r in rows:
        name = r["Kernel_Name"]
        if base_name(name) == "k_query_seed":
            seeds += 1
        if nb and seeds > nb and base_name(name).startswith("k_query"):
            continue
        out.setdefault(name, []).append(float(r["Counter_Value"]))
    return out


def main():
    docs, vocab, fdir, wdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    wanted = sys.argv[5:] or ["k_tok_fast", "k_agg_w", "k_rs_scatter", "k_query_win", "k_query_seed"]
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    res = {"docs": docs, "vocab": vocab,
           "method": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), mean over dispatches; separate --pmc passes; "
                     "kernels matched by exact base name (template instantiations summed per launch); "
                     "query kernels per batch (total / k_query_seed dispatches)",
           "kernels": {}}
    anchor = [v for n, v in fetch.items() if base_name(n) == "k_query_seed"]
    for k in wanted:
        fk = [v for n, v in fetch.items() if base_name(n) == k]
        wk = [v for n, v in write.items() if base_name(n) == k]
        if not fk or not wk:
            continue
        # template instantiations of one kernel are launched together: a "launch"
        # is the sum of their means.  A query kernel launched several times per
        # batch (k_query_win: window stages, overflow rounds) counts per batch:
        # total / k_query_seed dispatches
        if k.startswith("k_query") and anchor:
            nb = len(anchor[0])
            f = sum(sum(v) for v in fk) / nb * 1024
            w = sum(sum(v) for v in wk) / nb * 1024
        else:
            f = sum(sum(v) / len(v) for v in fk) * 1024
            w = sum(sum(v) / len(v) for v in wk) * 1024
        res["kernels"][k] = {"fetch_bytes_raw": round(f), "write_bytes": round(w),
                             "dispatches": sum(len(v) for v in fk), "instantiations": len(fk),
                             "batches": len(anchor[0]) if (k.startswith("k_query") and anchor) else None,
                             "hbm_bytes_per_launch": round(2 * f + w)}
    os.makedirs("profiles", exist_ok=True)
    # SME_PMC_OUT: e.g. profiles/pmc_traffic_c5.json for bench.py --config c5
    json.dump(res, open(os.environ.get("SME_PMC_OUT", "profiles/pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
