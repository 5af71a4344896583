#!/bin/bash
# Same-box A/B of library builds on the whole training step: rocprofv3 kernel trace of a
# short bench run per exp/*.so (ONEBIT_HIP_LIB), step windows into ab_<name>.txt.
# usage (gpurun, repo root): bash tools/gpu_ab_step.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for so in $R/exp/*.so; do
  n=$(basename $so .so)
  cd /tmp && ONEBIT_HIP_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $O/$n.log 2>&1 || exit 1
  python3 $R/tools/step_window.py $(ls $O/$n/run_kernel_trace.csv $O/$n/*/run_kernel_trace.csv 2>/dev/null | head -1) 60 > $O/ab_$n.txt || exit 1
done
