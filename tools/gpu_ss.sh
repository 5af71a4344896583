#!/bin/bash
# Subsampling session: its GPU tests + the model parity test, then a profiled short bench.
# usage (repo root, via gpurun): bash tools/gpu_ss.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-ss}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_subsample_gpu.py tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; grep '"metric"' $O/prof.log | cut -c1-300; exit $rc
