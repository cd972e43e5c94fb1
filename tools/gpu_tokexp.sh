# tokenizer timing experiments: SME_TOKEXP = 0 / 1 / 2 / 3 over tools/tok_experiment.py (V = 2^20 only)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for x in 0 1 2 3; do
  SME_TOKEXP=$x TOK_V=1048576 timeout -k 10 200 python3 tools/tok_experiment.py 250000 > gpurun_out/tokx_$x.log 2>&1 || { tail -5 gpurun_out/tokx_$x.log; exit 1; }
  echo "tokexp $x: $(grep '"V"' gpurun_out/tokx_$x.log | tail -1)"
done
