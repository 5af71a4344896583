#!/bin/bash
# Same-box A/B of the working tree against a baseline tree (e.g. `git archive HEAD` unpacked
# into ab_base/ and built there): the default bench line, alternating, N rounds.
# usage (GPU box, repo root): bash tools/gpu_ab_tree.sh TAG BASE_DIR [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
B=$2; N=${3:-2}
for i in $(seq $N); do
  for side in base new; do
    if [ $side = base ]; then D=$R/$B; else D=$R; fi
    (cd $D && timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 30) > $O/ab_${side}_$i.log 2>&1 || exit 1
    echo "$side run $i: $(tail -1 $O/ab_${side}_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
