#!/bin/bash
# The pmc_step.sh counter groups over any python tool (one rocprofv3 --pmc pass per group,
# kernel-trace only). usage (GPU box, repo root): bash tools/pmc_cmd.sh TAG tools/X.py [args]
# then: python tools/pmc_table.py gpurun_out/TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd /tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
G3="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
G4="FETCH_SIZE"
G5="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4" "$G5"; do
  i=$((i+1))
  echo "pass $i: $G"
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$O/p$i" -o pmc -- \
    python3 "$R/$1" "${@:2}" > "$O/p$i.log" 2>&1 || exit 1
done
