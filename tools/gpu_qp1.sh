# MaxScore seed-tile sweep (bench only): QP1="-1 0 4 8 16" values of SME_QP1, with SME_QSTATS counters
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for p in ${QP1:--1 0 4 8 16}; do
  SME_QSTATS=1 SME_QP1=$p timeout -k 10 300 python -u bench.py --cpu-docs 0 --steps 1 --warmup 1 "$@" > gpurun_out/bench_qp1_$p.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_qp1_$p.log; exit 1; }
  echo "p1 $p: $(grep -o '"ms_per_batch": [0-9.]*\|"kernel_ms": [0-9.]*\|"prep_ms": [0-9.]*\|query_sample_kernels_agree": [a-z]*' gpurun_out/bench_qp1_$p.log | tr '\n' ' ') $(grep SME_QSTATS gpurun_out/bench_qp1_$p.log | tail -1)"
done
