#!/bin/bash
# round 6: the overlapped deferred exchange -- tests, per-rank cost at world size 1 over RCCL,
# a kernel trace of the overlapped configuration
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python3 $R/tools/multi_path_bench.py 20 > $O/multi.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/tools/multi_path_bench.py 3 chunked > $O/prof.log 2>&1) || exit 1
echo done
