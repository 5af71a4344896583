#!/bin/bash
# One GPU-box session: GPU tests, bench (default line + torch-attention A/B), rocprof stats.
# usage (from the repo root, via gpurun): bash tools/gpu_run.sh TAG [skip-tests]
# A test run that ends in anything but pass/fail (rc > 1: crash, abort, timeout) stops it.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 300 python -m pytest tests/test_relattn_gpu.py -x -q > $O/relattn_tests.log 2>&1
  rc=$?; echo "relattn tests rc=$rc" >> $O/relattn_tests.log; [ $rc -gt 1 ] && exit $rc
  timeout -k 10 600 python -m pytest tests -m gpu -q > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/gpu_tests.log; [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 400 python bench.py --progress > $O/bench.log 2>&1 || exit 1
OB_ATTN=torch timeout -k 10 200 python bench.py --progress --no-cpu-baseline --no-roofline > $O/bench_torchattn.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1
