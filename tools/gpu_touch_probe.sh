# Does touching the device-resident dataset before the warmup change the driver-shaped window?
# usage (repo root, via gpurun): bash tools/gpu_touch_probe.sh
set -e
O=gpurun_out/touch
mkdir -p $O
for i in 1 2 3; do for T in 0 1; do
  DNN_BENCH_TOUCH=$T timeout -k 10 120 python bench.py --steps 20 --warmup 5 --diag-windows 2 > $O/b_${T}_$i.json 2> $O/b_${T}_$i.err
done; done
