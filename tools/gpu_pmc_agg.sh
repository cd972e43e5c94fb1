# PMC passes for the aggregation kernel (c2 build only): FETCH_SIZE, then L2 hits / misses
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmca_f $R/gpurun_out/pmca_h
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_agg_w|k_rs_scatter" --output-format csv -d $R/gpurun_out/pmca_f -o run -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-docs 0 --no-checks --no-query > $R/gpurun_out/pmca_f.log 2>&1 || { echo PMC_F_FAIL; tail -5 $R/gpurun_out/pmca_f.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_agg_w|k_rs_scatter" --output-format csv -d $R/gpurun_out/pmca_h -o run -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-docs 0 --no-checks --no-query > $R/gpurun_out/pmca_h.log 2>&1 || { echo PMC_H_FAIL; tail -5 $R/gpurun_out/pmca_h.log; exit 1; }
echo PMC_OK
