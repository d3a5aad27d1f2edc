# Rehearse the N-rank bench path with N ranks sharing ONE GPU (xGMI group of N regions on one
# device: exercises the 3/4-rank granule exchange, the self-tests, the votes and the timed
# loop).  (gloo for the host-side process group: RCCL refuses two ranks on one device)
# usage (from the repo root, via gpurun): bash tools/gpu_multirank.sh N [tag]
set -e
N=${1:-4}
T=${2:-b$N}
mkdir -p gpurun_out/mr
DNN_BACKEND=gloo OMP_NUM_THREADS=2 DNN_DEBUG_XGMI=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29731 bench.py --gpus $N --steps 300 --warmup 30 --no-epoch \
  > gpurun_out/mr/$T.json 2> gpurun_out/mr/$T.err
