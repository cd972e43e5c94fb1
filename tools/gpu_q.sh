set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "quer or smoke or forward" > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_q.log; exit $rc
