#!/bin/bash
# One GPU-box session. usage (via gpurun, repo root):
#   bash tools/gpu_session.sh TAG "TESTS" [bench] [prof] [pmc]
# steps: bench | prof | infer (configs[4] lines, int8 and fp32 activations) | pmc
# TESTS: pytest selection ("-" = none; "all" = every -m gpu test). Each step has its own
# time limit; the first failing step (rc > 1 for pytest: crash / abort / timeout) ends it.
set -o pipefail
export TMPDIR=/tmp
TAG=$1; TESTS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ "$TESTS" != "-" ]; then
  [ "$TESTS" = "all" ] && TESTS="tests -m gpu"
  timeout -k 10 900 python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/gpu_tests.log; [ $rc -gt 1 ] && exit $rc
fi
for step in "$@"; do
  case $step in
    bench) timeout -k 10 400 python bench.py --progress > $O/bench.log 2>&1 || exit 1 ;;
    prof) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1) || exit 1 ;;
    infer) timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline > $O/bench_infer_i8.log 2>&1 || exit 1
           timeout -k 10 300 python bench.py --mode infer-fp32act --no-cpu-baseline > $O/bench_infer_fp32act.log 2>&1 || exit 1 ;;
    pmc) bash $R/tools/pmc_step.sh $TAG/pmc > $O/pmc.log 2>&1 || exit 1 ;;
  esac
done
echo session done
