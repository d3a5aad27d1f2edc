# Layer-engine GPU tests + bench lines of every zoo model (+ a kernel trace of cifar-vgg bf16
# and lenet-bn fp32 for the per-layer dispatch table).   usage: bash tools/gpu_layers_bench.sh [outdir]
set -e
O=gpurun_out/${1:-lb}
mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
for m in "cifar-vgg bf16" "cifar-vgg fp32" "lenet-bn fp32" "lenet fp32"; do set -- $m
  timeout -k 10 300 python bench.py --model $1 --dtype $2 --engine layers --steps 300 --warmup 30 --no-epoch \
    > $O/b_$1_$2.json 2> $O/b_$1_$2.err
done
cd /tmp && export TMPDIR=/tmp
for m in "cifar-vgg bf16" "lenet-bn fp32"; do set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/p_$1_$2 -o run -- python3 $R/bench.py --model $1 --dtype $2 \
    --engine layers --steps 200 --warmup 20 --no-epoch > /dev/null 2>&1
done
