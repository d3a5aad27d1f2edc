# Per-layer dispatch table of the layer engine (cifar-vgg bf16, lenet-bn fp32) from a kernel trace.
# usage (repo root, via gpurun): bash tools/gpu_layers_table.sh [outdir]
set -e
O=gpurun_out/${1:-lt}
mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
for m in "cifar-vgg bf16" "lenet-bn fp32"; do set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/p_$1_$2 -o run -- python3 $R/bench.py --model $1 --dtype $2 \
    --engine layers --steps 200 --warmup 20 --no-epoch > $R/$O/b_$1_$2.json 2> $R/$O/b_$1_$2.err
done
