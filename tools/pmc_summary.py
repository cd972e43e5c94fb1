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
        if "k_query_seed" in name:
            seeds += 1
        if nb and seeds > nb and "k_query" in name:
            continue
        out.setdefault(name, []).append(float(r["Counter_Value"]))
    return out


def main():
    docs, vocab, fdir, wdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    wanted = sys.argv[5:] or ["k_tok_fast", "k_query"]
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    res = {"docs": docs, "vocab": vocab,
           "method": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), mean over dispatches; separate --pmc passes",
           "kernels": {}}
    for k in wanted:
        fk = [v for n, v in fetch.items() if k in n]
        wk = [v for n, v in write.items() if k in n]
        if not fk or not wk:
            continue
        # template instantiations of one kernel (e.g. the query kernel's register
        # and LDS paths) are launched together: a "launch" is the sum of their means
        # a kernel launched several times per batch (k_query_win: sample windows,
        # the rest, overflow rounds) counts per batch: total / k_query_seed dispatches
        anchor = [v for n, v in fetch.items() if "k_query_seed" in n] if "k_query_win" in k else []
        if anchor:
            nb = len(anchor[0])
            f = sum(sum(v) for v in fk) / nb * 1024
            w = sum(sum(v) for v in wk) / nb * 1024
        else:
            f = sum(sum(v) / len(v) for v in fk) * 1024
            w = sum(sum(v) / len(v) for v in wk) * 1024
        res["kernels"][k] = {"fetch_bytes_raw": round(f), "write_bytes": round(w), "dispatches": len(fk[0]),
                             "instantiations": len(fk), "hbm_bytes_per_launch": round(2 * f + w)}
    os.makedirs("profiles", exist_ok=True)
    json.dump(res, open("profiles/pmc_traffic.json", "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
