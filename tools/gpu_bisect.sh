#!/bin/bash
# Bisect a bench hang: small graph step, full-size eager, full-size graph, roofline alone.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-bisect}
mkdir -p $O
timeout -k 10 150 python bench.py --batch 8 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --progress > $O/b8_graph.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --batch 32 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --eager --progress > $O/b32_eager.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --batch 32 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --progress > $O/b32_graph.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --roofline-only --progress > $O/roofline.log 2>&1 || exit 1
