#!/bin/bash
# round 6: K-chunked dense GEMM (static A ring), CTC recursion ring, int8 absmax --
# tests, dense timings, the bench under rocprofv3 kernel stats, the inference lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/tools/dense_bench.py > $O/dense.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --steps 20 > $O/bench_prof.log 2>&1) || exit 1
timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline --no-roofline > $O/infer_i8.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode infer-fp32act --no-cpu-baseline --no-roofline > $O/infer_fp32act.log 2>&1 || exit 1
echo done
