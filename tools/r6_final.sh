#!/bin/bash
# round 6, final tree: PMC traffic of the roofline kernels (-> profiles/pmc_traffic.json),
# the default bench line (roofline + cpu_baseline), the bench under rocprofv3 kernel trace /
# stats (step window, roofline kernel duration), the int8 inference line's kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 bash $R/tools/traffic.sh $1/traffic > $O/traffic.log 2>&1 || exit 1
python3 $R/tools/traffic_json.py $O/traffic > $O/pmc_traffic.json 2> $O/traffic_json.err || exit 1
cp $O/pmc_traffic.json $R/profiles/pmc_traffic.json || exit 1
timeout -k 10 500 python bench.py > $O/benchfull.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/bench_prof.log 2>&1) || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_infer -o run -- python3 $R/bench.py --mode infer --no-cpu-baseline --no-roofline > $O/infer_prof.log 2>&1) || exit 1
rm -rf $O/traffic/*/  2>/dev/null
rm -f $O/prof_infer/run_kernel_trace.csv
echo done
