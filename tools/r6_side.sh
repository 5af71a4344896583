#!/bin/bash
# round 6: the finish tables beside the grouped dW launch -- tests, then the same-box bench A/B
# against deferred._SIDE_TABLES=False
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash $R/tools/ab_prof.sh $1/ab . "deferred._SIDE_TABLES=False" > $O/ab.log 2>&1 || exit 1
echo done
