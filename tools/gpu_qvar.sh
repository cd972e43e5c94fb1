# query-kernel env variants (bench only): QVAR="SME_QBM=0 SME_QBM=1,SME_QDENSE=128 ..." (comma joins vars of one run)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
i=0
for c in ${QVAR:-SME_QBM=0 SME_QBM=1}; do
  i=$((i+1))
  env $(echo $c | tr ',' ' ') timeout -k 10 300 python -u bench.py --cpu-docs 0 --steps 1 --warmup 1 --no-checks "$@" > gpurun_out/bench_qv_$i.log 2>&1 || { echo BENCH_FAIL $c; tail -30 gpurun_out/bench_qv_$i.log; exit 1; }
  echo "$c: $(grep -o '"ms_per_batch": [0-9.]*\|"prep_ms": [0-9.]*' gpurun_out/bench_qv_$i.log | tr '\n' ' ') $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench_qv_$i.log | tail -1)"
done
