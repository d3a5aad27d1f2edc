# Conv weight-gradient A/B: layer GPU tests, then the zoo bench lines with the LDS-patch wgrad
# (default) and the gather kernel (DNN_CONV_WGRAD=gather), plus a kernel trace of the default.
# usage (repo root, via gpurun): bash tools/gpu_wgrad_ab.sh [outdir]
set -e
O=gpurun_out/${1:-wab}
mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
for w in patch gather; do
  for m in "cifar-vgg bf16" "cifar-vgg fp32" "lenet-bn fp32" "lenet fp32"; do set -- $m
    DNN_CONV_WGRAD=$w timeout -k 10 300 python bench.py --model $1 --dtype $2 --engine layers --steps 300 --warmup 30 \
      --no-epoch > $O/b_${w}_$1_$2.json 2> $O/b_${w}_$1_$2.err
  done
done
cd /tmp && export TMPDIR=/tmp
for m in "cifar-vgg bf16" "lenet-bn fp32"; do set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/p_$1_$2 -o run -- python3 $R/bench.py --model $1 --dtype $2 \
    --engine layers --steps 200 --warmup 20 --no-epoch > /dev/null 2>&1
done
