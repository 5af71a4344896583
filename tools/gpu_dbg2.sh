#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-dbg2}
mkdir -p $O
timeout -k 10 200 python -u tools/debug_params.py > $O/params.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_layernorm_gpu.py tests/test_bitlinear_i8_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $O/tests.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --mode infer --progress > $O/bench_infer.log 2>&1 || exit 1
exit 0
