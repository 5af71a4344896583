#!/bin/bash
# Same-box per-kernel A/B: rocprofv3 kernel stats of the default bench line for the baseline
# tree, the working tree, and the working tree with a module switch set (python expression).
# usage (GPU box, repo root): bash tools/ab_prof.sh TAG BASE_DIR ["module.attr=value" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
B=$2; shift 2
run() {  # side dir [switch]
  local side=$1 dir=$2 sw=$3
  local pre="import sys, runpy; sys.argv=['bench.py','--no-cpu-baseline','--no-roofline','--steps','20']; sys.path.insert(0, '$dir/cmu-11785-idl-1.58bit-asr_amd')"
  if [ "${sw#env:}" != "$sw" ]; then  # env:NAME=VALUE (e.g. ONEBIT_HIP_LIB=exp/lib_x.so)
    pre="$pre; import os; os.environ['${sw#env:}'.split('=')[0]] = '$R/' + '${sw#env:}'.split('=', 1)[1]"
  elif [ -n "$sw" ]; then
    local mod=${sw%%.*} rest=${sw#*.}
    pre="$pre; from onebit_asr import $mod; $mod.${rest}"
  fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$side -o run -- python3 -c "$pre; import os; os.chdir('$dir'); runpy.run_path('$dir/bench.py', run_name='__main__')" > $O/$side.log 2>&1) || exit 1
  echo "$side: $(tail -1 $O/$side.log)"
}
run base $R/$B
run new $R
i=0
for sw in "$@"; do i=$((i+1)); run sw$i $R "$sw"; done
