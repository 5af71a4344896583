#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r1i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_relattn_gpu.py tests/test_bitlinear_gpu.py tests/test_bitlinear_passes_gpu.py tests/test_graph_step_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $O/tests.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python tools/attn_bench.py > $O/attn.log 2>&1 || exit 1
timeout -k 10 120 python tools/kbench.py > $O/kbench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --progress --no-cpu-baseline > $O/bench_train.log 2>&1 || exit 1
exit 0
