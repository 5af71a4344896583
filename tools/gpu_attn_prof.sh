#!/bin/bash
# attention kernels alone at the Conformer-S training shape: kernel stats + PMC limiter passes
# usage (GPU box, repo root): bash tools/gpu_attn_prof.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o attn -- python3 $R/tools/attn_bench.py --reps 10 > $O/stats.log 2>&1 || exit 1
bash $R/tools/pmc_attn.sh $1/pmc fwd > $O/pmc_fwd.log 2>&1 || exit 1
bash $R/tools/pmc_attn.sh $1/pmcb bwd > $O/pmc_bwd.log 2>&1 || exit 1
echo done
