# c4-shard build only, raw-table load factor variants: LOADS="40 60 80"
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for l in ${LOADS:-40 60 80}; do
  SME_RAWLOAD=$l timeout -k 10 400 python -u bench.py --config ${CFG:-c4shard} --steps 2 --warmup 1 --cpu-docs 0 --no-query --no-checks > gpurun_out/bench_c4l_$l.log 2>&1 || { echo FAIL $l; tail -20 gpurun_out/bench_c4l_$l.log; exit 1; }
  echo "load $l: $(python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stage_ms'];print(d['ms_per_step'],s['tok_kernel'],s['vocabulary'],s['aggregate'],s['sort_term'])" gpurun_out/bench_c4l_$l.log)"
done
