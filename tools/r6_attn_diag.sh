#!/bin/bash
# round 6: attention stamps (diagnostic builds exp/libstampK.so) + PMC groups over attn_bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for K in 3 2 4; do
  ONEBIT_HIP_LIB=$R/exp/libstamp$K.so timeout -k 10 120 python3 $R/tools/attn_stamps.py $K > $O/stamps$K.log 2>&1 || exit 1
done
timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 50 > $O/bench.log 2>&1 || exit 1
timeout -k 10 600 bash $R/tools/pmc_cmd.sh $1/pmc tools/attn_bench.py --reps 5 > $O/pmc.log 2>&1 || exit 1
if [ -n "$2" ]; then timeout -k 10 900 python -u -m pytest $2 -x -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || exit 1; fi
echo diag done
