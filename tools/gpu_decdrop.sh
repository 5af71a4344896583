#!/bin/bash
# Decoder residual dropout on the fused kernel: GPU tests, then a same-box step-time A/B of
# OB_DEC_RESDROP=0 (torch dropout + add) vs 1.
# usage (gpurun, repo root): bash tools/gpu_decdrop.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fused_gpu.py tests/test_layernorm_gpu.py tests/test_graph_step_gpu.py tests/test_conformer_s_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for f in 0 1; do
    OB_DEC_RESDROP=$f timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench_dd$f.$r.log 2>&1 || exit 1
    echo "OB_DEC_RESDROP=$f run $r: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_dd$f.$r.log)"
  done
done
