#!/bin/bash
# One GPU-box session: bench lines for the non-default configs (quant-off, inference).
# usage (from the repo root, via gpurun): bash tools/gpu_modes.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-modes}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python bench.py --mode quant-off --no-cpu-baseline --progress > $O/bench_quant_off.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline --progress > $O/bench_infer_i8.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode infer-fp32act --no-cpu-baseline --progress > $O/bench_infer_fp32act.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --conv-pw-ternary --no-cpu-baseline --progress > $O/bench_pw_ternary.log 2>&1 || exit 1
