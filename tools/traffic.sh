#!/bin/bash
# HBM traffic of the BitLinear kernels for bench.py's roofline "traffic" field: one
# rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE), kernel-trace only, over
# tools/kbench.py per (shape, op) and tools/dwg_bench.py (the grouped dW launch), eager
# launches (no graph replay under counters).
# usage (on the GPU box, repo root): bash tools/traffic.sh TAG
# then: python tools/traffic_json.py gpurun_out/TAG > profiles/pmc_traffic.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp
for shape in lin1 lin2 qkvo pos; do
  for op in fwd dx; do
    [ "$shape" = pos ] && [ "$op" = dx ] && continue
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$O/${shape}_${op}_${ctr}" -o pmc \
        -- python3 "$R/tools/kbench.py" --reps 5 --no-graph --shape $shape --op $op \
        > "$O/${shape}_${op}_${ctr}.log" 2>&1 || exit 1
    done
  done
done
# the grouped weight-gradient launch at the step's composition (tools/dwg_bench.py)
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/dwg_${ctr}" -o pmc \
    -- python3 "$R/tools/dwg_bench.py" --reps 3 --no-graph > "$O/dwg_${ctr}.log" 2>&1 || exit 1
done
echo traffic done
