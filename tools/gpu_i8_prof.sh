#!/bin/bash
# int8 GEMM alone: timing, kernel stats and one PMC group per pass. usage: bash tools/gpu_i8_prof.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 120 python3 $R/tools/i8bench.py > $O/time.log 2>&1 || exit 1
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/tools/i8bench.py --reps 5 > $O/stats.log 2>&1 || exit 1
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d $O/p$i -o pmc -- python3 $R/tools/i8bench.py --reps 2 > $O/p$i.log 2>&1 || exit 1
done
echo done
