#!/bin/bash
# round 6: query-side attention backward with each wave's dS' rows stored before dQu / dQv --
# parity tests, attention timings, the train bench under rocprofv3 stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/tools/attn_bench.py > $O/attn.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --steps 20 > $O/bench_prof.log 2>&1) || exit 1
rm -f $O/prof/run_kernel_trace.csv
echo done
