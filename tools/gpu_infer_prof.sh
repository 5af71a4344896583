set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-s2b}; mkdir -p $O
timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline > $O/bench_infer_i8.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_i8 -o run -- python3 $R/bench.py --mode infer --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $O/prof_i8.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f32 -o run -- python3 $R/bench.py --mode infer-fp32act --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $O/prof_f32.log 2>&1 || exit 1
echo done
