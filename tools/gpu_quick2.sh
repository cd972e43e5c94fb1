# GPU parity suite + a quick c2 bench line (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -10; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
SME_BENCH_VERBOSE=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --cpu-docs 0 > gpurun_out/bench_quick.log 2>&1; rc=$?
grep "query step walls" gpurun_out/bench_quick.log; tail -1 gpurun_out/bench_quick.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); q=d['query']
print('build', d['ms_per_step'], d['value'], 'tok', d['roofline']['kernel_ms'])
print('query', q['ms_per_batch'], q['value'], 'kernel', q['roofline']['kernel_ms'], q['kernel_split_ms'])
print('ser', d['stage_ms']['serialize_records_untimed']); print('e2e', d.get('end_to_end_ms'))"
exit $rc
