#!/bin/bash
# HBM traffic of the BitLinear kernels for bench.py's roofline "traffic" field: one
# rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE), kernel-trace only, over
# tools/kbench.py per (shape, op), eager launches (no graph replay under counters).
# usage (on the GPU box, repo root): bash tools/traffic.sh TAG
# then: python tools/traffic_json.py gpurun_out/TAG > profiles/pmc_traffic.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp
for shape in lin1 lin2 qkvo pos; do
  for op in fwd dx dw; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$O/${shape}_${op}_${ctr}" -o pmc \
        -- python3 "$R/tools/kbench.py" --reps 5 --no-graph --shape $shape --op $op \
        > "$O/${shape}_${op}_${ctr}.log" 2>&1 || exit 1
    done
  done
done
echo traffic done
