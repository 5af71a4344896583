#!/bin/bash
# End-of-session measurement: GPU tests, bench (default config), rocprofv3 kernel stats of
# the bench, then the PMC HBM-traffic passes for bench.py's roofline.traffic.
# usage (gpurun, repo root): bash tools/gpu_final.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_run.sh $1 || exit 1
bash $R/tools/traffic.sh $1_traffic || exit 1
