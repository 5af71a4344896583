#!/bin/bash
# Phase pricing: attention variants (exp/ra_*.so) via attn_bench, ternary-GEMM variants
# (exp/tg_*.so) via kbench --fused. usage (gpurun, repo root): bash tools/gpu_phases2.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for so in $R/exp/ra_*.so; do
  echo "== $(basename $so .so)" >> $O/phases.log
  ONEBIT_HIP_LIB=$so timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 30 >> $O/phases.log 2>&1 || exit 1
done
for so in $R/exp/tg_*.so; do
  echo "== $(basename $so .so)" >> $O/phases.log
  ONEBIT_HIP_LIB=$so timeout -k 10 180 python3 $R/tools/kbench.py --fused >> $O/phases.log 2>&1 || exit 1
done
