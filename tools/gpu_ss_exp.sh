#!/bin/bash
# Price the subsampling GEMM phases: rocprofv3 --stats of tools/ss_bench.py with the product
# library and each exp/ss_*.so variant (tools/variant.sh). usage: bash tools/gpu_ss_exp.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-ssexp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp
for v in base $(cd $R/exp && ls ss_*.so 2>/dev/null | sed 's/\.so$//'); do
  if [ $v = base ]; then unset ONEBIT_HIP_LIB; else export ONEBIT_HIP_LIB=$R/exp/$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python $R/tools/ss_bench.py --reps 5 > $O/$v.log 2>&1 || exit 1
  echo "$v: $(grep us/call $O/$v.log)"
done
