set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --model lenet --engine layers --dtype fp32 > gpurun_out/bl_lenet32.json 2> gpurun_out/bl1.err
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --model lenet-bn --dtype fp32 > gpurun_out/bl_bn32.json 2> gpurun_out/bl2.err
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --model cifar-vgg --dtype bf16 > gpurun_out/bl_vgg16.json 2> gpurun_out/bl3.err
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/b.json 2> gpurun_out/b.err
