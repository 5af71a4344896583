#!/bin/bash
# usage: bash tools/r6run.sh TAG "pytest selection" [bench] [benchfull] [prof] [attn] [dwg] [kbench]
# (round 6 GPU-call wrapper: each step under its own time limit, the call ends at the first failure)
set -o pipefail
TAG=$1; TESTS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
if [ "$TESTS" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS ${XFLAG--x} -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
fi
for st in "$@"; do case $st in
  bench) timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench.log 2>&1 || exit 1 ;;
  benchfull) timeout -k 10 400 python bench.py > $O/benchfull.log 2>&1 || exit 1 ;;
  dwg) timeout -k 10 300 python tools/dwg_bench.py > $O/dwg.log 2>&1 || exit 1 ;;
  attn) timeout -k 10 300 python tools/attn_bench.py > $O/attn.log 2>&1 || exit 1 ;;
  kbench) timeout -k 10 300 python tools/kbench.py --fused > $O/kbench.log 2>&1 || exit 1 ;;
  prof) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1) || exit 1 ;;
esac; done
echo done
