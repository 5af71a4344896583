#!/bin/bash
# LayerNorm A/B (tools/ln_bench.py, one process per setting): the tree's library vs
# ablib/old.so (a build of the previous layernorm.hip), then the launch-shape knobs.
# usage (GPU box, repo root): bash tools/gpu_ln_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for i in 1 2 3; do
  for lib in "$R/ablib/old.so" ""; do
    ONEBIT_HIP_LIB=$lib timeout -k 10 120 python tools/ln_bench.py >> $O/ln.jsonl 2>> $O/ln_err.log || exit 1
    tail -1 $O/ln.jsonl | cut -c1-200
  done
done
for cfg in "384 1" "256 1" "512 2"; do
  set -- $cfg
  OB_LN_BWD_BLOCKS=$1 OB_LN_RPT=$2 timeout -k 10 120 python tools/ln_bench.py >> $O/ln.jsonl 2>> $O/ln_err.log || exit 1
  tail -1 $O/ln.jsonl | cut -c1-200
done
# ternary GEMM grid size at K = 576 (lin2 fwd / fwd+residual): row tiles per block balance
for nb in 512 384 576 768 512; do
  echo "OB_TGEMM_BLOCKS=$nb" >> $O/tg.log
  OB_TGEMM_BLOCKS=$nb timeout -k 10 120 python tools/kbench.py --shape lin2 --fused --reps 50 >> $O/tg.log 2>&1 || exit 1
done
cat $O/tg.log
