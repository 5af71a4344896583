#!/bin/bash
# One GPU-box session: GPU tests, bench, rocprof kernel stats.
# usage (from the repo root, via gpurun): bash tools/gpu_run.sh TAG [skip-tests]
# A test run that ends in anything but pass/fail (rc > 1: crash, abort, timeout) stops it.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/gpu_tests.log; [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 400 python bench.py --progress > $O/bench.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
