# xGMI exchange forms on the one-GPU box: the xGMI GPU tests (1 rank: every form vs local SGD;
# 2 ranks: one-launch pull == two-launch == rsag bitwise), then 2 ranks sharing the GPU through
# bench.py with each form.  usage (repo root, via gpurun): bash tools/gpu_push.sh
set -e
O=gpurun_out/push
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
for X in pull rsag push; do
  DNN_XGMI_EXCHANGE=$X DNN_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29731 bench.py --gpus 2 --steps 1000 --warmup 50 \
    --no-epoch > $O/b2_$X.json 2> $O/b2_$X.err
done
