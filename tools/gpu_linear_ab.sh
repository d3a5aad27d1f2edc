# Linear-kernel A/B: layer GPU tests, then the zoo bench lines, plus cifar-vgg with every Linear
# on the MFMA kernels (DNN_LINEAR_MFMA_MAX raised above fc1's 67M MACs), with kernel traces.
# usage (repo root, via gpurun): bash tools/gpu_linear_ab.sh [outdir]
set -e
O=gpurun_out/${1:-lab}
mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
for m in "cifar-vgg bf16" "cifar-vgg fp32" "lenet-bn fp32" "lenet fp32"; do set -- $m
  timeout -k 10 300 python bench.py --model $1 --dtype $2 --engine layers --steps 300 --warmup 30 --no-epoch \
    > $O/b_$1_$2.json 2> $O/b_$1_$2.err
done
DNN_LINEAR_MFMA_MAX=1073741824 timeout -k 10 300 python bench.py --model cifar-vgg --dtype bf16 --engine layers \
  --steps 300 --warmup 30 --no-epoch > $O/b_mfma_cifar-vgg_bf16.json 2> $O/b_mfma_cifar-vgg_bf16.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/p_lenet_fp32 -o run -- python3 $R/bench.py --model lenet \
  --dtype fp32 --engine layers --steps 200 --warmup 20 --no-epoch > /dev/null 2>&1
DNN_LINEAR_MFMA_MAX=1073741824 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/p_mfma_vgg -o run -- python3 \
  $R/bench.py --model cifar-vgg --dtype bf16 --engine layers --steps 200 --warmup 20 --no-epoch > /dev/null 2>&1
