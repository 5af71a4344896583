#!/bin/bash
for nt in 12 9 6 4 3; do
  echo "NTMAX=$nt"; OB_TGEMM_NTMAX=$nt timeout -k 10 100 python tools/kbench.py --reps 30 2>&1 | grep -v amdgpu || exit 1
done
