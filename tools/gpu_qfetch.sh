# c2 query batch: timing (qexp) + one FETCH_SIZE pass and one TCC hit/miss pass over k_query_win
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/qexp.py --reps 3 $QARGS > gpurun_out/qf_time.log 2>&1 || { tail -5 gpurun_out/qf_time.log; exit 1; }
grep opts gpurun_out/qf_time.log | cut -c1-330
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/qf_fetch $R/gpurun_out/qf_tcc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_query_win" --output-format csv -d $R/gpurun_out/qf_fetch -o run -- python3 $R/tools/qexp.py --reps 0 $QARGS > $R/gpurun_out/qf_fetch.log 2>&1 || { echo FETCH_FAIL; tail -5 $R/gpurun_out/qf_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_query_win" --output-format csv -d $R/gpurun_out/qf_tcc -o run -- python3 $R/tools/qexp.py --reps 0 $QARGS > $R/gpurun_out/qf_tcc.log 2>&1 || { echo TCC_FAIL; tail -5 $R/gpurun_out/qf_tcc.log; exit 1; }
echo QF_OK
