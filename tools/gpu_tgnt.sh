set -o pipefail
mkdir -p gpurun_out/tgnt
for cfg in "12 512" "3 512" "3 1024" "4 1024" "6 768"; do
  set -- $cfg
  OB_TGEMM_NTMAX=$1 OB_TGEMM_BLOCKS=$2 timeout -k 10 120 python tools/kbench.py --reps 30 --fused > gpurun_out/tgnt/nt$1_b$2.log 2>&1 || exit 1
  echo "NTMAX=$1 BLOCKS=$2"; grep -A9 layer gpurun_out/tgnt/nt$1_b$2.log | grep -v layer | cut -c1-110
done
