#!/bin/bash
# A/B of BLAS routing on the bench step. usage: bash tools/blas_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $O/default.log 2>&1 || exit 1
OB_PW_BLAS=cublaslt timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $O/pw_lt.log 2>&1 || exit 1
OB_BLAS_ALL=cublas timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $O/all_rocblas.log 2>&1 || exit 1
