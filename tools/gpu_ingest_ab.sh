# Ingest folded into the first conv, A/B on one MI355X: the layer GPU tests, then the layer-engine
# benches with the first conv reading the u8 images itself (DNN_FUSE_INGEST=1) vs the ingest
# kernel (=0).  usage (repo root, via gpurun): bash tools/gpu_ingest_ab.sh
set -e
O=gpurun_out/ingest_ab
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_layers_gpu.py -x -v --timeout 120 --timeout-method thread \
  > $O/t.log 2>&1
for m in "lenet fp32" "cifar-vgg bf16" "lenet-bn fp32" "cifar-vgg fp32"; do set -- $m
  for f in 0 1; do
    DNN_FUSE_INGEST=$f timeout -k 10 300 python bench.py --model $1 --dtype $2 --engine layers --steps 300 \
      --warmup 30 --no-epoch > $O/b_$1_$2_f$f.json 2> $O/b_$1_$2_f$f.err
  done
done
