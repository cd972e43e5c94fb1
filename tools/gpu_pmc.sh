# PMC passes over a short bench run, one counter group per rocprofv3 run (kernel filter in $KRE)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
ARGS=${PMC_BENCH_ARGS:---docs 200000 --steps 1 --warmup 1 --no-query --cpu-docs 0}
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-.*}" -d $R/gpurun_out/pmc/p$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -5 $R/gpurun_out/pmc/p$i.log; exit 1; }
done
echo PMC_OK
