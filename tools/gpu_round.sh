set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_layers_gpu.py -m gpu -q > gpurun_out/tl.log 2>&1
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --model lenet-bn --dtype fp32 > gpurun_out/bl_bn32.json 2> gpurun_out/bl2.err
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --model cifar-vgg --dtype bf16 > gpurun_out/bl_vgg16.json 2> gpurun_out/bl3.err
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_bn -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-epoch --model lenet-bn --dtype fp32 > $R/gpurun_out/p_bn.log 2>&1
