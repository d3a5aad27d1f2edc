# Push vs pull forms of the xGMI exchange on the one-GPU box: the xGMI GPU tests (4-rank
# push == pull bitwise for the one-launch exchange, the two-launch kernel and the layer
# engine), then 4 ranks sharing the GPU through bench.py with each form.
# usage (repo root, via gpurun): bash tools/gpu_push.sh
set -e
O=gpurun_out/push
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
for X in push pull; do
  DNN_XGMI_EXCHANGE=$X DNN_BACKEND=gloo OMP_NUM_THREADS=2 DNN_DEBUG_XGMI=1 timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29731 bench.py --gpus 4 --steps 300 --warmup 30 \
    --no-epoch > $O/b4_$X.json 2> $O/b4_$X.err
  DNN_XGMI_EXCHANGE=$X DNN_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29733 bench.py --gpus 4 --steps 100 --warmup 10 \
    --no-epoch --engine layers --model cifar-vgg > $O/b4_vgg_$X.json 2> $O/b4_vgg_$X.err
done
