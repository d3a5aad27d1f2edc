set -e
# driver-shaped window (20/5): host wait mode A/B. HSA_ENABLE_INTERRUPT=0 makes ROCr poll
# completion signals instead of sleeping on an interrupt (the window ends in a device sync)
O=gpurun_out/${1:-r3s2_sync}
rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-epoch --diag-windows 2 > $O/def_$i.json 2> $O/def_$i.err
  HSA_ENABLE_INTERRUPT=0 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-epoch --diag-windows 2 > $O/poll_$i.json 2> $O/poll_$i.err
done
