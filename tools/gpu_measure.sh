# Round measurement: parity tests, smoke, bench line, kernel-trace stats, PMC traffic passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof $R/gpurun_out/pmc_f $R/gpurun_out/pmc_w
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-docs 0 --no-checks --no-e2e > $R/gpurun_out/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/bench_prof.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_tok_fast|k_query_win|k_query_seed" --output-format csv -d $R/gpurun_out/pmc_f -o run -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-docs 0 --no-checks --no-e2e > $R/gpurun_out/pmc_f.log 2>&1 || { echo PMC_F_FAIL; tail -5 $R/gpurun_out/pmc_f.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_tok_fast|k_query_win|k_query_seed" --output-format csv -d $R/gpurun_out/pmc_w -o run -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-docs 0 --no-checks --no-e2e > $R/gpurun_out/pmc_w.log 2>&1 || { echo PMC_W_FAIL; tail -5 $R/gpurun_out/pmc_w.log; exit 1; }
rm -rf $R/gpurun_out/pmc_sq
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "k_tok_fast|k_query_win" --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-docs 0 --no-checks --no-e2e > $R/gpurun_out/pmc_sq.log 2>&1 || { echo PMC_SQ_FAIL; tail -5 $R/gpurun_out/pmc_sq.log; exit 1; }
echo MEASURE_OK
