#!/bin/bash
# configs[4] inference, int8 and fp32 activations: bench lines + rocprofv3 kernel stats.
# usage (repo root, via gpurun): bash tools/gpu_infer.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp
for m in infer infer-fp32act; do
  timeout -k 10 300 python $R/bench.py --mode $m --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$m.log 2>&1 || exit 1
  grep metric $O/bench_$m.log | cut -c1-200
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python $R/bench.py --mode $m --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$m.log 2>&1 || exit 1
done
