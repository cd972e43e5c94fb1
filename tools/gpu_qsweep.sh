# query-kernel batch sweep: parity tests once, then the bench at each SME_QBATCH
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "quer" > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for b in ${QB:-4 8 16}; do
  SME_QBATCH=$b timeout -k 10 300 python -u bench.py --cpu-docs 0 --steps 1 --warmup 1 > gpurun_out/bench_q$b.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_q$b.log; exit 1; }
  echo "batch $b"; grep -o '"query": {[^}]*' gpurun_out/bench_q$b.log | cut -c1-200
done
