#!/bin/bash
# round 6: subsampling conv0 forward with 4 positions' windows in flight -- tests, timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/ss_bench.py > $O/ss.log 2>&1) || exit 1
rm -f $O/prof/run_kernel_trace.csv
echo done
