# kernel trace of the c2 build: per-build kernel time vs wall time (host-sync gaps)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/bgaps
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/bgaps -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-docs 0 --no-query --no-checks > $R/gpurun_out/bgaps/bench.log 2>&1 || { tail -5 $R/gpurun_out/bgaps/bench.log; exit 1; }
echo GAPS_OK
