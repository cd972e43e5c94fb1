# full default bench (build + c3 + checks + CPU baselines) -> gpurun_out/bench_full.log
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_full.log 2>&1; rc=$?
tail -2 gpurun_out/bench_full.log | cut -c1-6000; exit $rc
