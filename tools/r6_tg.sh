#!/bin/bash
# round 6: ternary-GEMM change -- tests, then same-box per-kernel A/B of the bench step (tree vs
# exp/libbase.so), then the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash $R/tools/ab_prof.sh $1/ab . env:ONEBIT_HIP_LIB=exp/libbase.so > $O/ab.log 2>&1 || exit 1
echo done
