#!/bin/bash
# Debug session: graph-vs-eager loss traces (stacked / literal, fused / torch optimizer),
# then the GPU test suite (no -x).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-dbg}
mkdir -p $O
timeout -k 10 200 python tools/debug_graph.py --mode graph > $O/graph.log 2>&1 || exit 1
timeout -k 10 200 python tools/debug_graph.py --mode graph --literal > $O/graph_literal.log 2>&1 || exit 1
timeout -k 10 200 python tools/debug_graph.py --mode graph --literal --torch-opt > $O/graph_literal_torchopt.log 2>&1 || exit 1
timeout -k 10 200 python tools/debug_graph.py --mode eager-gs > $O/eager_gs.log 2>&1 || exit 1
timeout -k 10 200 python tools/debug_graph.py --mode eager > $O/eager.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -q > $O/gpu_tests.log 2>&1
echo "tests rc=$?" >> $O/gpu_tests.log
