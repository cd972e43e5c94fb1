# raw-table load sweep (c2 build only): SME_RAWLOAD percent values
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for l in ${RL:-40 67 85}; do
  SME_RAWLOAD=$l timeout -k 10 300 python -u bench.py --cpu-docs 0 --steps 3 --warmup 2 --no-query --no-checks > gpurun_out/bench_rl_$l.log 2>&1 || { tail -5 gpurun_out/bench_rl_$l.log; exit 1; }
  echo "load $l: $(grep -o '"tok_kernel": [0-9.]*\|"vocabulary": [0-9.]*\|"total": [0-9.]*' gpurun_out/bench_rl_$l.log | tr '\n' ' ')"
done
