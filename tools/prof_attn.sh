#!/bin/bash
# Kernel stats of tools/attn_bench.py. usage: bash tools/prof_attn.sh TAG [attn_bench args]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift; mkdir -p $O
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/attn_bench.py "$@" > $O/prof.log 2>&1
