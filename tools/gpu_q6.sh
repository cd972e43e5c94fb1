# query parity subset, qexp variants, one SQ PMC pass
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/qpmc
bash tools/gpu_q5.sh || exit $?
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/qpmc/sq -o sq --output-format csv -- python3 $R/tools/qexp.py --reps 1 > $R/gpurun_out/qpmc/sq.log 2>&1
