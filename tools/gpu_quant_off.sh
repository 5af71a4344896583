set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/s2n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -2 $O/gpu_tests.log
for m in train quant-off quant-off-lib; do timeout -k 10 300 python bench.py --mode $m --no-cpu-baseline --no-roofline --steps 20 > $O/bench_$m.log 2>&1 || exit 1; echo "$m $(tail -1 $O/bench_$m.log | cut -c1-160)"; done
