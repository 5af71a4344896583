#!/bin/bash
# Same-box A/B of library builds with tools/attn_bench.py: bash tools/gpu_ab_attn_lib.sh TAG lib.so
# (the in-tree library, then the given one, twice each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; LIB=$2
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 50 > $O/tree_$rep.log 2>&1 || exit 1
  ONEBIT_HIP_LIB=$R/$LIB timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 50 > $O/lib_$rep.log 2>&1 || exit 1
done
echo ab done
