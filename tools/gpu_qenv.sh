# query-kernel env sweep (bench only): QENV="D:B D:B ..." = SME_QDENSE:SME_QBATCH pairs
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for c in ${QENV:-0:8 0:4 8:4 8:8 2:8 32:8}; do
  d=${c%%:*}; b=${c##*:}
  SME_QDENSE=$d SME_QBATCH=$b timeout -k 10 300 python -u bench.py --cpu-docs 0 --steps 1 --warmup 1 > gpurun_out/bench_qe_${d}_${b}.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_qe_${d}_${b}.log; exit 1; }
  echo "dense $d batch $b: $(grep -o '"ms_per_batch": [0-9.]*\|"kernel_ms": [0-9.]*\|"prep_ms": [0-9.]*' gpurun_out/bench_qe_${d}_${b}.log | tr '\n' ' ')"
done
