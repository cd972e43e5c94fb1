# query-path parity tests (+ dist), then tools/qexp.py variants and a quick bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_dist_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK:-quer or forward or repl or scale or dist or c2_full}" > gpurun_out/pytest_q.log 2>&1; rc=$?
grep -E "FAILED|ERROR|Error" gpurun_out/pytest_q.log | head -20; tail -3 gpurun_out/pytest_q.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/qexp.py --opts "${QOPTS:-query_kernel=2;seed_m=0;seed_m=256;cand_cap=256}" > gpurun_out/qexp.log 2>&1; rc=$?
cut -c1-400 gpurun_out/qexp.log
exit $rc
