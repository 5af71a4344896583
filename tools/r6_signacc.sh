#!/bin/bash
# round 6: sign-accumulate A/B (timing + PMC), dense GEMM timing, a pytest selection, the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python3 $R/tools/signacc_ab.py > $O/signacc.log 2>&1 || exit 1
timeout -k 10 120 python3 $R/tools/dense_bench.py > $O/dense.log 2>&1 || exit 1
timeout -k 10 600 bash $R/tools/pmc_cmd.sh $1/pmc tools/signacc_ab.py --reps 5 > $O/pmc.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench.log 2>&1 || exit 1
echo done
