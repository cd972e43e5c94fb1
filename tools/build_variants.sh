# Build A/B variants of libsme for kernel experiments (never the product): each
# variant recompiles one source (default sme_query.hip; name@file.hip picks another)
# with its own -D flags and links it with the product's other objects into
# simple-mapreduce-search-engine-information-retrieval-_amd/libsme_<name>.so.
#   VARIANTS="w4:-DSME_QWIN_WAVES=4 tok4@sme_build.hip:-DSME_TOKG=4,-DSME_NT=1" bash tools/build_variants.sh
# (several -D flags of one variant separated by commas)
# A variant named base-<rev> builds sme_query.hip as of git revision <rev>.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/simple-mapreduce-search-engine-information-retrieval-_amd
make -s -C $P >/dev/null
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function -Wno-unused-variable -Wno-unused-result"
for v in $VARIANTS; do
  name=${v%%:*}; defs=${v#*:}; [ "$defs" = "$v" ] && defs=""; defs=${defs//,/ }
  file=sme_query.hip
  case $name in *@*) file=${name#*@}; name=${name%%@*};; esac
  OTHERS=$(ls $P/build/*.o | grep -v "/${file%.hip}.o")
  mkdir -p $P/build_var/$name
  src=$P/csrc/$file
  case $name in base-*) src=$P/csrc/_var_query_${name#base-}.hip; git -C $R show ${name#base-}:simple-mapreduce-search-engine-information-retrieval-_amd/csrc/sme_query.hip > $src;; esac
  /opt/rocm/bin/hipcc $FLAGS $defs -c $src -o $P/build_var/$name/${file%.hip}.o
  case $name in base-*) rm -f $src;; esac
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $P/libsme_$name.so $OTHERS $P/build_var/$name/${file%.hip}.o
  echo "built libsme_$name.so ($defs)"
done
