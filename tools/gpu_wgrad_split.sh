# conv weight-gradient split sweep (workgroup target / slice cap / chunks per slice) on the zoo
# models' layer-engine step.  usage (repo root, via gpurun): bash tools/gpu_wgrad_split.sh [outdir]
set -e
O=gpurun_out/${1:-wsplit}
mkdir -p $O
for cfg in "1024 256 4" "1024 512 2" "2048 512 2" "2048 1024 1" "512 256 4"; do set -- $cfg
  for m in "lenet fp32" "lenet-bn fp32" "cifar-vgg bf16"; do set -- $cfg $m
    DNN_WGRAD_WGS=$1 DNN_WGRAD_MAX_SLICES=$2 DNN_WGRAD_MIN_CHUNKS=$3 timeout -k 10 200 python bench.py --model $4 \
      --dtype $5 --engine layers --steps 300 --warmup 30 --no-epoch > $O/b_$1_$2_$3_$4_$5.json 2> $O/b_$1_$2_$3_$4_$5.err
  done
done
