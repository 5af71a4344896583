set -o pipefail
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_relattn_gpu.py tests/test_fused_gpu.py tests/test_conformer_s_oracle_gpu.py tests/test_model_gpu.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "rc=$?" >> $O/tests.log
timeout -k 10 120 python tools/attn_bench.py --reps 20 > $O/attn.log 2>&1
