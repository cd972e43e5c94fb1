# GPU test suite (QK: -k filter), c2 qexp, c5 qexp (1M top-100)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${QK:+-k "$QK"} > gpurun_out/pytest_q.log 2>&1; rc=$?
grep -E "FAILED|Error" gpurun_out/pytest_q.log | head; tail -1 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/qexp.py --reps 2 > gpurun_out/qexp_c2.log 2>&1 || exit 1
cut -c1-330 gpurun_out/qexp_c2.log | tail -1
timeout -k 10 500 python -u tools/qexp.py --config c5 --docs 8841823 --queries 1000000 --k 100 --reps 1 ${C5OPTS:+--opts "$C5OPTS"} > gpurun_out/qexp_c5.log 2>&1; rc=$?
cut -c1-330 gpurun_out/qexp_c5.log | tail -4; exit $rc
