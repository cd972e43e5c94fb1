# query kernel counters (experiment build, SME_QSTATS) and part-switch timings (SME_QEXP)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export SME_LIB_PATH=$GRAFT_REPO_ROOT/simple-mapreduce-search-engine-information-retrieval-_amd/libsme_exp.so
for e in ${QEXPS:-0 1 2}; do
  SME_QLDS=${QLDS:-0} SME_QSTATS=${QSTATS:-0} SME_QEXP=$e timeout -k 10 400 python -u tools/qexp.py --reps 1 $QARGS > gpurun_out/qexp_$e.log 2>&1 || { tail -5 gpurun_out/qexp_$e.log; exit 1; }
  echo "== QEXP=$e"; grep -E "SME_QSTATS|opts" gpurun_out/qexp_$e.log | tail -3 | cut -c1-300
done
