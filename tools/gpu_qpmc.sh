# PMC passes over one c3 batch (tools/qexp.py, default path): SQ stall split and
# instruction mix, L2 hit/miss, HBM fetch -- each pass its own rocprofv3 run
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/qpmc; cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() { timeout -k 10 240 rocprofv3 --pmc $2 -d $R/gpurun_out/qpmc/$1 -o $1 --output-format csv -- python3 $R/tools/qexp.py --reps 1 --queries ${NQ:-100000} > $R/gpurun_out/qpmc/$1.log 2>&1; }
run sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" && \
run sq2 "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" && \
run tcc "TCC_HIT_sum TCC_MISS_sum" && \
run fetch "FETCH_SIZE"
rc=$?
find $R/gpurun_out/qpmc -name "*counter_collection.csv" | head; exit $rc
