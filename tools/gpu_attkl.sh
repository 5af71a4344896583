#!/bin/bash
# Fused decoder losses: GPU parity tests (their own + the full-size stacked-vs-literal step),
# then a same-box step-time A/B of OB_ATT_KL=0 (torch expressions) vs 1 (csrc/seqloss.hip).
# usage (gpurun, repo root): bash tools/gpu_attkl.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_seqloss_gpu.py tests/test_conformer_s_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for f in 0 1; do
    OB_ATT_KL=$f timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench_attkl$f.$r.log 2>&1 || exit 1
    echo "OB_ATT_KL=$f run $r: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_attkl$f.$r.log)"
  done
done
