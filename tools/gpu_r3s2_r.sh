set -e
# layer engine, cifar-vgg: library GEMM for the big fc1 (default) vs the hand-written MFMA GEMMs
# everywhere (DNN_LINEAR_MFMA_MAX raised), bf16 and fp32 layer modes
O=gpurun_out/${1:-r3s2_r}
rm -rf $O; mkdir -p $O
for dt in bf16 fp32; do
  timeout -k 10 200 python bench.py --model cifar-vgg --engine layers --dtype $dt --steps 300 --warmup 30 --no-epoch > $O/vgg_${dt}_lib.json 2> $O/vgg_${dt}_lib.err
  DNN_LINEAR_MFMA_MAX=1000000000 timeout -k 10 200 python bench.py --model cifar-vgg --engine layers --dtype $dt --steps 300 --warmup 30 --no-epoch > $O/vgg_${dt}_mfma.json 2> $O/vgg_${dt}_mfma.err
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DNN_LINEAR_MFMA_MAX=1000000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mfma -o run -- python3 bench.py --model cifar-vgg --engine layers --dtype bf16 --steps 300 --warmup 30 --no-epoch > $O/prof_mfma.log 2>&1
