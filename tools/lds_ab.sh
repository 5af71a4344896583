#!/bin/bash
# A/B: register-streamed ternary GEMM vs the opt-in LDS-staged one (OB_TGEMM_LDS=1)
timeout -k 10 100 python tools/kbench.py --reps 30 --fused 2>&1 | grep -v amdgpu || exit 1
echo "--- OB_TGEMM_LDS=1"
OB_TGEMM_LDS=1 timeout -k 10 100 python tools/kbench.py --reps 30 --fused 2>&1 | grep -v amdgpu || exit 1
