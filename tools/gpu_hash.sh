set -o pipefail
mkdir -p gpurun_out/hash
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_relattn_gpu.py tests/test_graph_step_gpu.py tests/test_stacked_step_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hash/tests.log 2>&1; rc=$?; tail -2 gpurun_out/hash/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/kbench.py --reps 30 --fused > gpurun_out/hash/kbench.log 2>&1 && grep fused gpurun_out/hash/kbench.log | head -2
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hash/attn -o run -- python3 $GRAFT_REPO_ROOT/tools/attn_bench.py --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/hash/attn.log 2>&1
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/hash/bench.log 2>&1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/hash/bench.log
