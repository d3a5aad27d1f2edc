# Layer-engine check on one MI355X: kernel tests, per-model bench lines, one kernel profile.
# usage (from the repo root, via gpurun): bash tools/gpu_layers.sh
set -e
mkdir -p gpurun_out/pl
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py tests/test_engine_gpu.py -k "layer or conv" -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/pl/t.log 2>&1
for m in "cifar-vgg bf16" "cifar-vgg fp32" "lenet-bn fp32" "lenet fp32"; do set -- $m
  timeout -k 10 300 python bench.py --model $1 --dtype $2 --engine layers --steps 300 --warmup 30 --no-epoch \
    > gpurun_out/pl/b_$1_$2.json 2>gpurun_out/pl/b_$1_$2.err
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pl/p_vgg_bf16 -o run -- \
  python3 $R/bench.py --model cifar-vgg --dtype bf16 --engine layers --steps 200 --warmup 20 --no-epoch > /dev/null 2>&1
