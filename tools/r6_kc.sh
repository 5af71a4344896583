#!/bin/bash
# round 6: long-K dense GEMM -- tests, timing against the library fp32 GEMM, bench step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/tools/dense_bench.py > $O/dense.log 2>&1 || exit 1
timeout -k 10 900 bash $R/tools/ab_prof.sh $1/ab . env:ONEBIT_HIP_LIB=exp/libhead.so > $O/ab.log 2>&1 || exit 1
echo done
