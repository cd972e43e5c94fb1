# query-path parity tests + quick c2 bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "quer or forward or repl or smoke" > gpurun_out/pytest_q.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_q.log | tail -20; tail -3 gpurun_out/pytest_q.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-docs 0 "$@" > gpurun_out/bench_quick.log 2>&1; rc=$?
tail -3 gpurun_out/bench_quick.log | cut -c1-4000; exit $rc
