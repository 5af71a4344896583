#!/bin/bash
# Attention kernels alone (tools/attn_bench.py): the working tree's library vs a baseline
# tree's (BASE_DIR, e.g. ab_base/ = git archive HEAD, built), alternating, N rounds.
# usage (GPU box, repo root): bash tools/gpu_ab_attn_tree.sh TAG BASE_DIR [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
B=$R/$2/cmu-11785-idl-1.58bit-asr_amd/onebit_asr/libonebit_hip.so; N=${3:-2}
for i in $(seq $N); do
  for lib in "$B" ""; do
    echo "== ${lib:-tree} run $i" >> $O/ab.log
    ONEBIT_HIP_LIB=$lib timeout -k 10 120 python3 $R/tools/attn_bench.py --reps 30 >> $O/ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/ab.log
