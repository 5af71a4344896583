#!/bin/bash
# Focused GPU check: selected test files first (stop on crash), then the full GPU suite
# and a bench line. usage: bash tools/gpu_quick.sh TAG "tests/test_a.py tests/test_b.py" [bench]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; FILES=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest $FILES -m gpu -v --timeout 120 --timeout-method thread > $O/focus.log 2>&1
rc=$?; echo "focus rc=$rc" >> $O/focus.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/gpu_tests.log; [ $rc -gt 1 ] && exit $rc
if [ "$3" == "bench" ]; then
  timeout -k 10 400 python bench.py --progress --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
fi
