#!/bin/bash
# int8-activation vs bf16x3 (fp32-exact) BitLinear forward: per-kernel times at the training
# and inference row counts, plus one PMC pass (MFMA busy, HBM fetch) per kernel at lin1.
# usage (from the repo root, via gpurun): bash tools/gpu_i8.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-i8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python $R/tools/kbench.py --i8 > $O/kbench_i8_train.log 2>&1 || exit 1
timeout -k 10 200 python $R/tools/kbench.py --i8 --passes 1 --rows 63744 > $O/kbench_i8_infer.log 2>&1 || exit 1
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE FETCH_SIZE --output-format csv -d $O/pmc_fwd -o pmc -- python3 $R/tools/kbench.py --i8 --passes 1 --rows 63744 --shape lin1 --op fwd --reps 10 > $O/pmc_fwd.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE FETCH_SIZE --output-format csv -d $O/pmc_fwd_i8 -o pmc -- python3 $R/tools/kbench.py --i8 --passes 1 --rows 63744 --shape lin1 --op fwd_i8 --reps 10 > $O/pmc_fwd_i8.log 2>&1 || exit 1
