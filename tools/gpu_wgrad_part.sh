# conv weight-gradient split: cap on the slice-partial bytes per layer (DNN_WGRAD_MAX_PART_KB)
# on the zoo models' layer-engine step.  usage (repo root, via gpurun): bash tools/gpu_wgrad_part.sh [outdir]
set -e
O=gpurun_out/${1:-wpart}
mkdir -p $O
for kb in 1073741824 8192 4096 2048 1024 512; do
  for m in "cifar-vgg bf16" "cifar-vgg fp32" "lenet-bn fp32" "lenet fp32"; do set -- $kb $m
    DNN_WGRAD_MAX_PART_KB=$1 timeout -k 10 200 python bench.py --model $2 \
      --dtype $3 --engine layers --steps 300 --warmup 30 --no-epoch > $O/b_$1_$2_$3.json 2> $O/b_$1_$2_$3.err
  done
done
