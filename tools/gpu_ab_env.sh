#!/bin/bash
# Same-box A/B of an environment switch on the default bench line.
# usage (GPU box, repo root): bash tools/gpu_ab_env.sh TAG VAR "A_VALUE B_VALUE" [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
VAR=$2; VALS=$3; N=${4:-2}
for i in $(seq $N); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 30 > $O/ab_${v}_$i.log 2>&1 || exit 1
    echo "$VAR=$v run $i: $(tail -1 $O/ab_${v}_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
