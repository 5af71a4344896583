#!/bin/bash
# same-box A/B of the decoder/CTC branch streams: bench with and without, twice each
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 --branch-streams > $O/branch_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 > $O/single_$i.log 2>&1 || exit 1
done
for f in $O/branch_*.log $O/single_*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
