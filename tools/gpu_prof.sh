#!/bin/bash
# rocprofv3 kernel stats of one bench mode: bash tools/gpu_prof.sh TAG MODE [extra bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; MODE=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$MODE -o run -- python3 $R/bench.py --mode $MODE --steps 3 --warmup 1 --no-cpu-baseline --no-roofline "$@" > $O/prof_$MODE.log 2>&1
