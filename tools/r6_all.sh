#!/bin/bash
# round 6, final tree in one call: the whole GPU suite, smoke(), PMC traffic of the roofline
# kernels (-> profiles/pmc_traffic.json), the default bench line, the bench under rocprofv3
# kernel trace / stats, the int8 inference line's kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
bash $R/tools/r6_final.sh $1 || exit 1
echo all done
