#!/bin/bash
# round 6: dense GEMM parity tests and timings
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/tools/dense_bench.py > $O/dense.log 2>&1 || exit 1
echo done
