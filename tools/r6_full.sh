#!/bin/bash
# round 6: the whole GPU suite, a same-box per-kernel A/B against exp/libbase.so, the full bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash $R/tools/ab_prof.sh $1/ab . env:ONEBIT_HIP_LIB=exp/libbase.so > $O/ab.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > $O/benchfull.log 2>&1 || exit 1
echo done
