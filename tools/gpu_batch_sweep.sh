# Per-GPU batch sweep of the headline engine on one MI355X: one bench line per batch size (the
# reference's run_training.sh sweep bs 1..64, extended to the sizes that fill all 256 CUs).
# usage (repo root, via gpurun): bash tools/gpu_batch_sweep.sh [outdir]
set -e
O=gpurun_out/${1:-bsweep}
mkdir -p $O
for bs in 1 4 16 64 128 256 512 1024; do
  timeout -k 10 200 python bench.py --batch-size $bs --steps 2000 --warmup 200 > $O/b_$bs.json 2> $O/b_$bs.err
  echo "bs=$bs done"
done
