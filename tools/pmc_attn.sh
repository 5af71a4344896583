#!/bin/bash
# PMC passes over tools/attn_bench.py (one rocprofv3 --pmc pass per group).
# usage: bash tools/pmc_attn.sh TAG OP
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
OP=$2
mkdir -p $O
cd /tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
G5="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES TCC_HIT_sum TCC_MISS_sum"
i=0
for G in "$G1" "$G2" "$G3" "$G4" "$G5"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d "$O/p$i" -o pmc -- python3 "$R/tools/attn_bench.py" --reps 3 --op $OP > "$O/p$i.log" 2>&1 || exit 1
done
echo pmc done
