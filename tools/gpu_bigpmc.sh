# FETCH_SIZE / WRITE_SIZE passes (one counter group per rocprofv3 run) of the c5 and
# c4-shard bench runs -> gpurun_out/pmc_{f,w}_{c5,c4shard}; then, here, e.g.
#   SME_PMC_BATCHES=2 SME_PMC_OUT=profiles/pmc_traffic_c5.json python tools/pmc_summary.py 8841823 30000 gpurun_out/pmc_f_c5 gpurun_out/pmc_w_c5
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
KRE=${KRE:-"k_tok_fast|k_agg_w|k_rs_scatter|k_query_win|k_query_seed"}
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-c5 c4shard}; do
  for p in f:FETCH_SIZE w:WRITE_SIZE; do
    d=$R/gpurun_out/pmc_${p%%:*}_$c; rm -rf $d
    timeout -s KILL 500 rocprofv3 --pmc ${p#*:} --kernel-include-regex "$KRE" --output-format csv -d $d -o run -- python3 $R/bench.py --config $c --steps 1 --warmup 1 --cpu-docs 0 --no-e2e > $d.log 2>&1 || { echo PMC_FAIL $c $p; tail -5 $d.log; exit 1; }
  done
done
echo BIGPMC_OK
