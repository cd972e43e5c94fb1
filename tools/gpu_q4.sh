# full GPU suite, then query-kernel experiments (tools/qexp.py) on the product
# library and on the experiment build (SME_QSTATS counters)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
PKGD=$GRAFT_REPO_ROOT/simple-mapreduce-search-engine-information-retrieval-_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -15; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/qexp.py --opts "${QOPTS:-seed_tiles=0;seed_tiles=8;heavy_div=0;heavy_div=8;query_order=0;query_kernel=1}" > gpurun_out/qexp.log 2>&1; rc=$?
cat gpurun_out/qexp.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
SME_LIB_PATH=$PKGD/libsme_exp.so SME_QSTATS=1 timeout -k 10 300 python -u tools/qexp.py --reps 1 --opts "${QOPTS2:-seed_tiles=0;heavy_div=0}" > gpurun_out/qexp_stats.log 2>&1; rc=$?
grep -v "^$" gpurun_out/qexp_stats.log | cut -c1-300 | tail -20; exit $rc
