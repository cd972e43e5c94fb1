# GPU experiment runner (run through gpurun from the repo root):
#   TESTS="none" | "" (all -m gpu tests) | "<pytest -k expression>"
#   BENCH="<bench.py args>"   (empty: no bench)
#   LIBS="libsme.so libsme_g4.so"   (library variants under the package dir, each benched)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
PKG=simple-mapreduce-search-engine-information-retrieval-_amd
if [ "${TESTS:-}" != "none" ]; then
  K=(); [ -n "${TESTS:-}" ] && K=(-k "$TESTS")
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
[ -z "${BENCH:-}" ] && exit 0
for L in ${LIBS:-libsme.so}; do
  echo "== $L"
  SME_LIB_PATH=$GRAFT_REPO_ROOT/$PKG/$L timeout -k 10 400 python -u bench.py $BENCH > gpurun_out/bench_$L.log 2>&1 \
    || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$L.log; exit 1; }
  tail -1 gpurun_out/bench_$L.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('ms_per_step', d['ms_per_step'], 'value', d['value'])
print('stage_ms', {k:v for k,v in d.get('stage_ms',{}).items() if not isinstance(v,dict)})
q=d.get('query')
if q: print('query', q.get('value'), q.get('ms_per_batch'), q.get('kernel_split_ms'), q.get('roofline',{}).get('kernel_ms'))
print('checks', d.get('checks'))
"
done
