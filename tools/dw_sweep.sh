#!/bin/bash
for s in 8 16; do
  echo "DW_MAXSTEPS=$s"; OB_DW_MAXSTEPS=$s timeout -k 10 100 python tools/kbench.py --reps 30 --op dw 2>&1 | grep -v amdgpu || exit 1
done
