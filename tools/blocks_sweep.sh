#!/bin/bash
for b in 512 1024 2048 100000; do
  echo "BLOCKS=$b"; OB_TGEMM_BLOCKS=$b timeout -k 10 100 python tools/kbench.py --reps 30 --fused 2>&1 | grep -v amdgpu || exit 1
done
