#!/bin/bash
# Debug session: new-kernel tests, then a long graph-mode run printing every step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-dbg}
mkdir -p $O
timeout -k 10 200 python -m pytest tests/test_embedding_gpu.py tests/test_relattn_gpu.py -x -q > $O/new_tests.log 2>&1
rc=$?; echo "rc=$rc" >> $O/new_tests.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 240 python tools/debug_graph.py --mode graph --batch 32 --steps 16 > $O/graph_b32.log 2>&1 || exit 1
