# A/B of libsme variants (tools/build_variants.sh) on one c2 / c3 batch (tools/qexp.py):
# kernel ms, wall ms, and a digest of every docno / score bit (must agree across
# variants).  LIBS="w4 w5" QARGS="..." bash tools/gpu_variants.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/var
for v in ${LIBS}; do
  SME_LIB_PATH=$R/simple-mapreduce-search-engine-information-retrieval-_amd/libsme_$v.so timeout -k 10 300 python3 -u tools/qexp.py --reps ${REPS:-3} $QARGS > gpurun_out/var/$v.log 2>&1 || { echo VAR_FAIL $v; tail -5 gpurun_out/var/$v.log; exit 1; }
  grep opts gpurun_out/var/$v.log | cut -c1-330
done
echo VARIANTS_OK
