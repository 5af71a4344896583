set -o pipefail
mkdir -p gpurun_out/tg4
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_bitlinear_gpu.py tests/test_bitlinear_passes_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tg4/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tg4/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/kbench.py --reps 30 --fused > gpurun_out/tg4/kbench.log 2>&1 && cat gpurun_out/tg4/kbench.log | head -12
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tg4/bench.log 2>&1; grep metric gpurun_out/tg4/bench.log | cut -c1-250
