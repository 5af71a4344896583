#!/bin/bash
# One GPU-box session: GPU tests, bench (graph + eager), rocprof kernel stats of the bench.
# usage (from the repo root, via gpurun): bash tools/gpu_run.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/gpu_tests.log 2>&1
echo "tests rc=$?" >> $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_graph.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --eager > $O/bench_eager.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1
