#!/bin/bash
# rocprofv3 kernel trace + stats of the default (graph-mode) bench step.
# usage: bash tools/gpu_prof_step.sh TAG [extra bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline "$@" > $O/prof.log 2>&1
