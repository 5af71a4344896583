set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
for m in 128 1024 8192 23904; do
  timeout -k 10 120 python tools/dense_bench.py --m $m --iters 50 > $O/dense_m$m.log 2>&1 || exit 1
done
for r in 128 1024 23904; do
  timeout -k 10 120 python tools/kbench.py --shape qkvo --rows $r --passes 1 --fused > $O/kb_qkvo_r$r.log 2>&1 || exit 1
done
echo ok
