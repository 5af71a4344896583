#!/bin/bash
# Price kernel phases: rocprofv3 --stats of one bench script with the product library and
# with each exp/PREFIX*.so variant (tools/variant.sh). usage (repo root, via gpurun):
#   bash tools/gpu_exp.sh TAG PREFIX tools/attn_bench.py [args...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; PREFIX=$2; SCRIPT=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp
for v in base $(cd $R/exp && ls ${PREFIX}*.so 2>/dev/null | sed 's/\.so$//'); do
  if [ $v = base ]; then unset ONEBIT_HIP_LIB; else export ONEBIT_HIP_LIB=$R/exp/$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/$SCRIPT "$@" > $O/$v.log 2>&1 || exit 1
  echo "$v done"
done
