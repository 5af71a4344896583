#!/bin/bash
# attention kernels alone at the Conformer-S training shape: timing, kernel stats and the
# PMC limiter passes (tools/pmc_run.sh; table: python tools/pmc_table.py gpurun_out/TAG/pmc 1)
# usage (GPU box, repo root): bash tools/gpu_attn_prof.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 20 > $O/time.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o attn -- python3 $R/tools/attn_bench.py --reps 10 > $O/stats.log 2>&1) || exit 1
bash $R/tools/pmc_run.sh $O/pmc python3 $R/tools/attn_bench.py --reps 3 > $O/pmc.log 2>&1 || exit 1
echo done
