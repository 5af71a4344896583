#!/bin/bash
# round 6: int8 lin1 launches with the next row tile's A in flight -- tests, the int8
# inference line under rocprofv3 stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_infer -o run -- python3 $R/bench.py --mode infer --no-cpu-baseline --no-roofline > $O/infer_prof.log 2>&1) || exit 1
rm -f $O/prof_infer/run_kernel_trace.csv
echo done
