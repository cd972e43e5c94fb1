# Round measurement on one GPU, in two gpurun calls (each under gpurun's 20-minute cap):
#   PART=a  parity tests (-m gpu), smoke(), the default bench line -> gpurun_out/{pytest_gpu,smoke,bench}.log
#   PART=b  rocprofv3 kernel-trace stats of a c2 bench run (checks + serializer included), then separate
#           PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run) over the build, serializer and
#           query kernels -> gpurun_out/{prof,pmc_f,pmc_w}; then, here,
#           SME_PMC_BATCHES=40 python tools/pmc_summary.py 1000000 1048576 gpurun_out/pmc_f gpurun_out/pmc_w
#           writes profiles/pmc_traffic.json (the first 40 query batches are the headline c3 ones)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
if [ "${PART:-a}" = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
  timeout -k 10 900 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log | cut -c1-400
  echo MEASURE_A_OK
  exit 0
fi
KRE=${KRE:-"k_tok_fast|k_agg_w|k_rs_scatter|k_rs_count|k_vocab|k_tfsort|k_tf_tile|k_ser_write|k_ser_big|k_query_win|k_query_seed"}
BARGS="--steps 1 --warmup 1 --cpu-docs 0 --no-e2e"
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof $R/gpurun_out/pmc_f $R/gpurun_out/pmc_w
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-docs 0 --no-e2e > $R/gpurun_out/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/bench_prof.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $R/gpurun_out/pmc_f -o run -- python3 $R/bench.py $BARGS > $R/gpurun_out/pmc_f.log 2>&1 || { echo PMC_F_FAIL; tail -5 $R/gpurun_out/pmc_f.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $R/gpurun_out/pmc_w -o run -- python3 $R/bench.py $BARGS > $R/gpurun_out/pmc_w.log 2>&1 || { echo PMC_W_FAIL; tail -5 $R/gpurun_out/pmc_w.log; exit 1; }
echo MEASURE_B_OK
