#!/bin/bash
# round 6: long-K dense GEMM + the int8 absmax launch -- tests, timings, bench-step A/B against
# exp/libhead.so, the int8 / fp32-activation inference lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/tools/dense_bench.py > $O/dense.log 2>&1 || exit 1
timeout -k 10 900 bash $R/tools/ab_prof.sh $1/ab . env:ONEBIT_HIP_LIB=exp/libhead.so > $O/ab.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline --no-roofline > $O/infer_i8.log 2>&1 || exit 1
ONEBIT_HIP_LIB=$R/exp/libhead.so timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline --no-roofline > $O/infer_i8_head.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode infer-fp32act --no-cpu-baseline --no-roofline > $O/infer_fp32act.log 2>&1 || exit 1
echo done
