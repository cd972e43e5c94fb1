# full GPU test suite, then a quick c2 bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -15; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-docs 0 > gpurun_out/bench_quick.log 2>&1; rc=$?
tail -2 gpurun_out/bench_quick.log | cut -c1-5000; exit $rc
