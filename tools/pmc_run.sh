#!/bin/bash
# Limiter counter passes over any program (one rocprofv3 --pmc pass per counter group,
# kernel-trace only); the output dirs p1..p5 are what tools/pmc_table.py reads.
# usage (GPU box): bash tools/pmc_run.sh OUTDIR python3 script.py args...
set -o pipefail
O=$1; shift
mkdir -p $O
cd /tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
G3="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
G4="FETCH_SIZE"
G5="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4" "$G5"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$O/p$i" -o pmc -- "$@" > "$O/p$i.log" 2>&1 || exit 1
done
echo pmc done
