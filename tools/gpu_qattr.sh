# k_query_win attribution: the experiment build's part switches
# (SME_QEXP, timing only -- results are wrong by design) on one c2 / c3 batch, each
# timed (tools/qexp.py) and measured with its own PMC pass ($PMC, default FETCH_SIZE;
# e.g. PMC="FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" -- one pass, within the
# per-block counter limits):
#   0  full kernel
#   2  no exact candidate scoring (tf bytes, LDS / global tf search, list appends)
#   3  also no passing-block impact sums (heavy impact rows)
#   7  also no sparse postings (docno / tf of the window, LDS sums)
#  15  also no heavy block bounds (bmq rows): records, skip entries, pipeline only
# QARGS passes e.g. "--config c5 --docs 8841823 --queries 1000000 --k 100".
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/qattr
export SME_LIB_PATH=$R/simple-mapreduce-search-engine-information-retrieval-_amd/libsme_exp.so
cd /tmp && export TMPDIR=/tmp
for e in ${QEXPS:-0 2 3 7 15}; do
  SME_QEXP=$e timeout -k 10 300 python3 -u $R/tools/qexp.py --reps 2 $QARGS > $R/gpurun_out/qattr/time_$e.log 2>&1 || { echo TIME_FAIL $e; tail -5 $R/gpurun_out/qattr/time_$e.log; exit 1; }
  echo "== QEXP=$e $(grep opts $R/gpurun_out/qattr/time_$e.log | tail -1 | cut -c1-200)"
  rm -rf $R/gpurun_out/qattr/f_$e
  SME_QEXP=$e timeout -s KILL 300 rocprofv3 --pmc ${PMC:-FETCH_SIZE} --kernel-include-regex "k_query_win" --output-format csv -d $R/gpurun_out/qattr/f_$e -o run -- python3 $R/tools/qexp.py --reps 0 $QARGS > $R/gpurun_out/qattr/f_$e.log 2>&1 || { echo FETCH_FAIL $e; tail -5 $R/gpurun_out/qattr/f_$e.log; exit 1; }
done
echo QATTR_OK
