# SQ counters of k_tok_fast over tools/tok_experiment.py (V = 64 / 2^14 / 2^20)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/tokprof
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "k_tok_fast" -d $R/gpurun_out/tokprof/p$i -o run --output-format csv -- python3 $R/tools/tok_experiment.py 250000 > $R/gpurun_out/tokprof/p$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -5 $R/gpurun_out/tokprof/p$i.log; exit 1; }
done
echo TOKPROF_OK
