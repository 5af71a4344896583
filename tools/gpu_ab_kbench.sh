#!/bin/bash
# A/B of library builds: tools/kbench.py --fused against every exp/*.so.
# usage (gpurun, repo root): bash tools/gpu_ab_kbench.sh TAG [kbench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift; mkdir -p $O
for so in $R/exp/*.so; do
  echo "== $(basename $so .so)" >> $O/ab.log
  ONEBIT_HIP_LIB=$so timeout -k 10 180 python3 $R/tools/kbench.py --fused "$@" >> $O/ab.log 2>&1 || exit 1
done
