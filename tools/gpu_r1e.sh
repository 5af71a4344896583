#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r1e}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_layernorm_gpu.py tests/test_graph_step_gpu.py -v --timeout 120 --timeout-method thread > $O/tests_a.log 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_a.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_bitlinear_i8_gpu.py tests/test_graph_step_gpu.py -v --timeout 120 --timeout-method thread > $O/tests_b.log 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_b.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --mode infer --conv-find --progress --no-roofline > $O/bench_infer_find.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode train --conv-find --progress --no-roofline --no-cpu-baseline > $O/bench_train_find.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode train --progress --no-roofline --no-cpu-baseline > $O/bench_train.log 2>&1 || exit 1
exit 0
