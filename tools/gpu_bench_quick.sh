# quick bench: build + c3 query batch, no CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-docs 0 "$@" > gpurun_out/bench_quick.log 2>&1; rc=$?
tail -3 gpurun_out/bench_quick.log | cut -c1-3000; exit $rc
