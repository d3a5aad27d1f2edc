# Layer-engine kernel tests + conv micro-benchmarks + the vgg bf16 / lenet fp32 bench lines.
# usage (from the repo root, via gpurun): bash tools/gpu_layers_quick.sh
set -e
mkdir -p gpurun_out/pq
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pq/t.log 2>&1
: > gpurun_out/pq/micro.txt
for cfg in "fwd 64 32 32 32 3 1 1" "fwd 64 64 16 64 3 1 1" "dgrad 64 32 32 32 3 1 1" "fwd 64 3 32 6 5 0 0" "fwd 64 32 32 32 3 1 0"; do
  timeout -k 10 120 python tools/conv_micro.py $cfg 200 >> gpurun_out/pq/micro.txt 2>&1
done
for m in "cifar-vgg bf16" "lenet fp32" "cifar-vgg fp32"; do set -- $m
  timeout -k 10 300 python bench.py --model $1 --dtype $2 --engine layers --steps 300 --warmup 30 --no-epoch \
    > gpurun_out/pq/b_$1_$2.json 2>gpurun_out/pq/b_$1_$2.err
done
