#!/bin/bash
# Time tools/attn_bench.py under each exp/ra_*.so variant. usage: bash tools/ra_variants.sh TAG [op]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
OPARG=${2:+--op $2}
for f in $R/exp/ra_*.so; do
  n=$(basename $f .so)
  echo "== $n" >> $O/variants.log
  ONEBIT_HIP_LIB=$f timeout -k 10 60 python $R/tools/attn_bench.py $OPARG >> $O/variants.log 2>&1 || exit 1
done
