#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-dbg3}
mkdir -p $O
timeout -k 10 200 python -u tools/debug_params.py --warm > $O/params_warm.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_relattn_gpu.py -v --timeout 120 --timeout-method thread > $O/relattn.log 2>&1
rc=$?; echo "rc=$rc" >> $O/relattn.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --mode train --progress --no-cpu-baseline --no-roofline > $O/bench_train.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_train -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $GRAFT_REPO_ROOT/$O/prof_train.log 2>&1
exit 0
