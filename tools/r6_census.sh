#!/bin/bash
# round 6: where the step's copies / fills come from (torch.profiler census of one eager step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python3 $R/tools/copy_census.py > $O/census.log 2>&1 || exit 1
echo done
