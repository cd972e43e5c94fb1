# c5 (8.84 M passages, 1 M top-100 queries) and c4 shard (6.25 M docs) on one GPU -> profiles/r04_bench_{c5,c4shard}.json
# CPU5 / CPU4: the bench's CPU-leg arguments for each (default: no CPU legs)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config c5 --steps 2 --warmup 1 ${CPU5:---cpu-docs 0} --no-e2e > gpurun_out/bench_c5.log 2>&1 || { echo C5_FAIL; tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-300
timeout -k 10 500 python -u bench.py --config c4shard --steps 2 --warmup 1 ${CPU4:---cpu-docs 0} --no-e2e > gpurun_out/bench_c4shard.log 2>&1 || { echo C4_FAIL; tail -20 gpurun_out/bench_c4shard.log; exit 1; }
tail -1 gpurun_out/bench_c4shard.log | cut -c1-300
echo BIG_OK
