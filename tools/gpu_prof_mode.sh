#!/bin/bash
# kernel trace + stats of a short bench run in one mode. usage: bash tools/gpu_prof_mode.sh TAG MODE
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --mode $2 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1
