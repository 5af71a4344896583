#!/bin/bash
# q/k/v dW finishes grouped in one launch: GPU tests, then a same-box step-time A/B of
# OB_DW_GROUP=0 (one finish launch per layer) vs 1.
# usage (gpurun, repo root): bash tools/gpu_dwgroup.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fused_gpu.py tests/test_bitlinear_passes_gpu.py tests/test_graph_step_gpu.py tests/test_conformer_s_gpu.py tests/test_abi_cpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for f in 0 1; do
    OB_DW_GROUP=$f timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench_dwg$f.$r.log 2>&1 || exit 1
    echo "OB_DW_GROUP=$f run $r: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_dwg$f.$r.log)"
  done
done
