# tokenizer timing split (experiment build libsme_x.so, SME_TOKEXP switches; wrong
# results by design, so no checks): c2 build stage times per switch
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
PKG=simple-mapreduce-search-engine-information-retrieval-_amd
for X in ${XS:-0 1 2 4 8}; do
  SME_TOKEXP=$X SME_LIB_PATH=$GRAFT_REPO_ROOT/$PKG/libsme_x.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 \
    --cpu-docs 0 --no-query --no-e2e --no-checks > gpurun_out/tokx_$X.log 2>&1 || { echo FAIL $X; tail -20 gpurun_out/tokx_$X.log; exit 1; }
  tail -1 gpurun_out/tokx_$X.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('TOKEXP=$X', 'tok', s['tok_kernel'], 'total', s['total'])"
done
