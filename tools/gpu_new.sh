#!/bin/bash
# Focused GPU session: the given test files first, then optional bench modes.
# usage: bash tools/gpu_new.sh TAG "tests/a.py tests/b.py" "mode1 mode2 ..."
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-new}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest $2 -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -gt 1 ] && exit $rc
fi
for m in $3; do
  timeout -k 10 300 python bench.py --mode $m --progress --no-cpu-baseline > $O/bench_$m.log 2>&1 || exit 1
done
exit 0
