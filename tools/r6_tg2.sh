#!/bin/bash
# round 6: per-kernel A/B of the bench step -- tree, exp/lib_kw2.so, exp/lib_kw4.so, exp/libbase.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
if [ -n "$2" ]; then timeout -k 10 900 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1; fi
timeout -k 10 1000 bash $R/tools/ab_prof.sh $1/ab . env:ONEBIT_HIP_LIB=exp/lib_kw2.so env:ONEBIT_HIP_LIB=exp/lib_kw4.so env:ONEBIT_HIP_LIB=exp/libbase.so > $O/ab.log 2>&1 || exit 1
echo done
