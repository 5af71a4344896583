#!/bin/bash
# Kernel stats of tools/attn_bench.py under each exp/ra_*.so. usage: bash tools/ra_prof_variants.sh TAG [bench args]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift; mkdir -p $O
for f in $R/exp/ra_*.so; do
  n=$(basename $f .so)
  cd /tmp && ONEBIT_HIP_LIB=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $R/tools/attn_bench.py --reps 5 "$@" > $O/$n.log 2>&1 || exit 1
done
