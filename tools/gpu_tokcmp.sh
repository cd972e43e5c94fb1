# build-step timing: product library vs the experiment library (SME_LIB_PATH)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "build or kat or fuzz" > gpurun_out/pytest_b.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_b.log; [ $rc -eq 0 ] || exit $rc
for L in libsme.so libsme_exp.so; do
  SME_LIB_PATH=$GRAFT_REPO_ROOT/simple-mapreduce-search-engine-information-retrieval-_amd/$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-docs 0 --no-query --no-e2e > gpurun_out/bench_$L.log 2>&1 || { tail -5 gpurun_out/bench_$L.log; exit 1; }
  tail -1 gpurun_out/bench_$L.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['ms_per_step'], 'tok', d['roofline']['kernel_ms'], d['stage_ms']['aggregate'], d['checks'].get('sum_tf_eq_tokens'))"
done
