#!/bin/bash
# Kernel-trace stats of tools/attn_bench.py for the in-tree library and, if given, another
# build: bash tools/gpu_prof_attn.sh TAG [lib.so]   -> gpurun_out/TAG/{tree,lib}/run_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tree -o run -- python3 $R/tools/attn_bench.py --reps 20 > $O/prof_tree.log 2>&1 || exit 1
if [ -n "$2" ]; then
  export ONEBIT_HIP_LIB=$R/$2
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lib -o run -- python3 $R/tools/attn_bench.py --reps 20 > $O/prof_lib.log 2>&1 || exit 1
fi
echo prof done
