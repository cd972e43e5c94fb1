# tokenizer timing variants over tools/tok_experiment.py (env per variant, TVARS="A=1;B=2")
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
IFS=';' read -ra VS <<< "DEFAULT=1;$TVARS"
for v in "${VS[@]}"; do
  echo "== $v"
  env $v timeout -k 10 200 python -u tools/tok_experiment.py ${TOKN:-250000} 2>&1 | grep '^{' | cut -c1-200 || exit 1
done
