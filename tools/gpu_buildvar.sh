# A/B of libsme variants on the c2 build step (bench.py without queries / CPU legs /
# checks): ms per step and the per-stage device times.  LIBS="cur tr4" bash tools/gpu_buildvar.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/bvar
for v in ${LIBS}; do
  SME_LIB_PATH=$R/simple-mapreduce-search-engine-information-retrieval-_amd/libsme_$v.so timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-10} --warmup 2 --no-query --cpu-docs 0 --no-e2e --no-checks $BARGS > gpurun_out/bvar/$v.log 2>&1 || { echo BVAR_FAIL $v; tail -5 gpurun_out/bvar/$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bvar/$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], {k: d['stage_ms'][k] for k in ('tok_kernel','tokenize','vocabulary','aggregate','sort_term','sort_tf') if k in d['stage_ms']})"
done
echo BUILDVAR_OK
