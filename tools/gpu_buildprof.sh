# kernel-trace stats of the c2 build only (no query batch, no CPU baseline)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/buildprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/buildprof -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-docs 0 --no-query --no-checks "$@" > $R/gpurun_out/buildprof/bench.log 2>&1 || { tail -5 $R/gpurun_out/buildprof/bench.log; exit 1; }
f=$(find $R/gpurun_out/buildprof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:-float(r["TotalDurationNs"]))
for r in rows[:45]:
    print("%-60s %6s %10.3f ms avg %8.3f ms" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"])/1e6, float(r["AverageNs"])/1e6))
PY
