# query kernel profile: stats counters + PMC FETCH / WRITE / SQ passes on the c3 batch
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/qprof
SME_QSTATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-docs 0 > gpurun_out/qprof/bench.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/qprof/bench.log; exit 1; }
grep SME_QSTATS gpurun_out/qprof/bench.log | tail -2
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "k_query_imp" -d $R/gpurun_out/qprof/p$i -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-docs 0 > $R/gpurun_out/qprof/p$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -5 $R/gpurun_out/qprof/p$i.log; exit 1; }
done
echo QPROF_OK
