set -e
# 2 ranks time-sharing the one GPU (host collectives over gloo; RCCL refuses 2 ranks per GPU):
# the multi-GPU bench path end to end with its start-up all-reduce A/B, bf16 and fp32
O=gpurun_out/${1:-r3s2_q}
rm -rf $O; mkdir -p $O
DNN_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29701 bench.py --gpus 2 --steps 200 --warmup 20 > $O/bench2_bf16.json 2> $O/bench2_bf16.err
DNN_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 --steps 200 --warmup 20 --dtype fp32 > $O/bench2_fp32.json 2> $O/bench2_fp32.err
