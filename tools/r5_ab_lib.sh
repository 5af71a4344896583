#!/bin/bash
# same-box A/B: kbench of the in-tree library vs exp/*.so libraries, twice each
# usage: bash tools/r5_ab_lib.sh TAG "kbench args" exp/libX.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; ARGS=$2; shift 2
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 150 python3 $R/tools/kbench.py $ARGS > $O/base_$rep.log 2>&1 || exit 1
  for lib in "$@"; do
    n=$(basename $lib .so)
    ONEBIT_HIP_LIB=$R/$lib timeout -k 10 150 python3 $R/tools/kbench.py $ARGS > $O/${n}_$rep.log 2>&1 || exit 1
  done
done
echo ab done
