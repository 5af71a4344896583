#!/bin/bash
# Phase pricing of the attention kernels: tools/attn_bench.py against every exp/ra_*.so
# variant (built by tools/variant.sh with one RA_/RB_/RK_EXP_ switch each).
# usage (gpurun, repo root): bash tools/gpu_attn_phases.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for so in $R/exp/ra_*.so; do
  n=$(basename $so .so)
  echo "== $n" >> $O/phases.log
  ONEBIT_HIP_LIB=$so timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 30 >> $O/phases.log 2>&1 || exit 1
done
