#!/bin/bash
# round 6: same-box A/B of the in-tree library against exp/libbase.so (attn_bench, dense_bench,
# twice each), then an optional pytest selection and the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 50 > $O/attn_tree_$rep.log 2>&1 || exit 1
  ONEBIT_HIP_LIB=$R/exp/libbase.so timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 50 > $O/attn_base_$rep.log 2>&1 || exit 1
  timeout -k 10 120 python3 $R/tools/dense_bench.py > $O/dense_tree_$rep.log 2>&1 || exit 1
  ONEBIT_HIP_LIB=$R/exp/libbase.so timeout -k 10 120 python3 $R/tools/dense_bench.py > $O/dense_base_$rep.log 2>&1 || exit 1
done
if [ -n "$2" ]; then timeout -k 10 900 python -u -m pytest $2 -x -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || exit 1; fi
if [ -n "$3" ]; then timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench.log 2>&1 || exit 1; fi
echo ab done
