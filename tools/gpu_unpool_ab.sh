# Unpooling data gradient A/B on one MI355X: the layer GPU tests, then the layer-engine lenet
# bench with the dgrad reading the pooled gradient (DNN_UNPOOL_DGRAD=1) vs relu_pool_bwd + the
# plain dgrad (=0), plus a kernel trace of the new path.  usage: bash tools/gpu_unpool_ab.sh
set -e
O=gpurun_out/unpool_ab
mkdir -p $O
R=$PWD
timeout -k 10 500 python -u -m pytest tests/test_layers_gpu.py -x -v --timeout 120 --timeout-method thread \
  > $O/t.log 2>&1
for rep in 1 2; do for u in 0 1; do
  DNN_UNPOOL_DGRAD=$u timeout -k 10 300 python bench.py --model lenet --dtype fp32 --engine layers --steps 300 \
    --warmup 30 --no-epoch > $O/b_u${u}_r$rep.json 2> $O/b_u${u}_r$rep.err
done; done
DNN_UNPOOL_DGRAD=1 timeout -k 10 300 python bench.py --model lenet --dtype bf16 --engine layers --steps 300 \
  --warmup 30 --no-epoch > $O/b_bf16_u1.json 2> $O/b_bf16_u1.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
  python3 $R/bench.py --model lenet --dtype fp32 --engine layers --steps 200 --warmup 20 --no-epoch > /dev/null 2>&1
