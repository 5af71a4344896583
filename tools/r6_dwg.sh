#!/bin/bash
# round 6: grouped-dW work order -- tests, per-kernel A/B of the bench step against exp/libhead.so,
# the grouped launch alone (dwg_bench), PMC FETCH/WRITE of the grouped launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 $R/tools/dwg_bench.py > $O/dwg_tree.log 2>&1 || exit 1
ONEBIT_HIP_LIB=$R/exp/libhead.so timeout -k 10 300 python3 $R/tools/dwg_bench.py > $O/dwg_head.log 2>&1 || exit 1
timeout -k 10 900 bash $R/tools/ab_prof.sh $1/ab . env:ONEBIT_HIP_LIB=exp/libhead.so > $O/ab.log 2>&1 || exit 1
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o pmc -- python3 $R/tools/dwg_bench.py --no-graph --reps 3 > $O/pmc_$C.log 2>&1 || exit 1
done
echo done
