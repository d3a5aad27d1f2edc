# Push vs pull form of the one-launch xGMI exchange on the one-GPU box: the xGMI GPU tests
# (incl. the 4-rank push == pull bitwise test), then N ranks sharing the GPU through bench.py
# with each form.  usage (repo root, via gpurun): bash tools/gpu_push.sh
set -e
O=gpurun_out/push
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
for N in 4 8; do for X in push pull; do
  DNN_XGMI_EXCHANGE=$X DNN_BACKEND=gloo OMP_NUM_THREADS=2 DNN_DEBUG_XGMI=1 timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29731 bench.py --gpus $N --steps 300 --warmup 30 \
    --no-epoch > $O/b${N}_$X.json 2> $O/b${N}_$X.err
done; done
