# query parity tests + quick bench with query stats
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "quer or forward" > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
SME_QSTATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-docs 0 "$@" > gpurun_out/bench_q.log 2>&1 || { tail -5 gpurun_out/bench_q.log; exit 1; }
grep SME_QSTATS gpurun_out/bench_q.log | tail -1
python3 -c "
import json; l=[x for x in open('gpurun_out/bench_q.log') if x.startswith('{')][-1]; d=json.loads(l)
q=d['query']; print('build ms', d['ms_per_step'], 'query ms/batch', q['ms_per_batch'], 'kernel', q['roofline']['kernel_ms'], 'prep', q['prep_ms'], 'QPS', q['value'])"
if [ -n "$QALT" ]; then
env $QALT SME_QSTATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-docs 0 > gpurun_out/bench_q2.log 2>&1 || { tail -5 gpurun_out/bench_q2.log; exit 1; }
echo "ALT $QALT"; grep SME_QSTATS gpurun_out/bench_q2.log | tail -1
python3 -c "
import json; l=[x for x in open('gpurun_out/bench_q2.log') if x.startswith('{')][-1]; d=json.loads(l)
q=d['query']; print('build ms', d['ms_per_step'], 'query ms/batch', q['ms_per_batch'], 'kernel', q['roofline']['kernel_ms'], 'prep', q['prep_ms'], 'QPS', q['value'])"
fi
