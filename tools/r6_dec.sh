#!/bin/bash
# round 6: decoder attention backward in two launches, embedding backward prefetch --
# parity tests, the decoder-attention bench, the train bench under rocprofv3 stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/tools/decattn_bench.py > $O/decattn.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --steps 20 > $O/bench_prof.log 2>&1) || exit 1
echo done
