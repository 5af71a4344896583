#!/bin/bash
# A/B of library builds on the attention kernels: tools/attn_bench.py against exp/*.so,
# then the GPU test suite and the default bench on the in-tree library.
# usage (gpurun, repo root): bash tools/gpu_ab_attn.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for so in $R/exp/*.so; do
  echo "== $(basename $so .so)" >> $O/ab.log
  ONEBIT_HIP_LIB=$so timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 30 >> $O/ab.log 2>&1 || exit 1
done
