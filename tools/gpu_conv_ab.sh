# Layer-engine conv A/B: GPU layer tests, then cifar-vgg bf16 / fp32 and lenet fp32 bench lines
# with the patch kernel's subtile count forced to 1 and 2 (DNN_CONV_NSUB), plus per-layer
# dispatch tables of the default plan.   usage (repo root, via gpurun): bash tools/gpu_conv_ab.sh [outdir]
set -e
O=gpurun_out/${1:-cab}
mkdir -p $O
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
for ns in 1 2; do
  for m in "cifar-vgg bf16" "cifar-vgg fp32" "lenet-bn fp32"; do set -- $m
    DNN_CONV_NSUB=$ns timeout -k 10 300 python bench.py --model $1 --dtype $2 --engine layers --steps 300 --warmup 30 \
      --no-epoch > $O/b_ns${ns}_$1_$2.json 2> $O/b_ns${ns}_$1_$2.err
  done
done
cd /tmp && export TMPDIR=/tmp
for m in "cifar-vgg bf16" "lenet-bn fp32"; do set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/p_$1_$2 -o run -- python3 $R/bench.py --model $1 --dtype $2 \
    --engine layers --steps 200 --warmup 20 --no-epoch > /dev/null 2>&1
done
