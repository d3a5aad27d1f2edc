# Rehearse the N-rank bench path with N ranks sharing ONE GPU (xGMI group of N regions on one
# device: exercises the 4/8-rank flag layout, the exchange self-test, the vote and the timed
# loop).  FENCES=3 forces the fence set that groups spanning several GPUs use.
# (gloo for the host-side process group: RCCL refuses two ranks on one device)
# usage (from the repo root, via gpurun): [FENCES=3] bash tools/gpu_multirank.sh N [tag]
set -e
N=${1:-4}
T=${2:-b$N}
mkdir -p gpurun_out/mr
[ -n "$FENCES" ] && export DNN_XGMI_FENCES=$FENCES
DNN_BACKEND=gloo OMP_NUM_THREADS=2 DNN_DEBUG_XGMI=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29731 bench.py --gpus $N --steps 300 --warmup 30 --no-epoch \
  > gpurun_out/mr/$T.json 2> gpurun_out/mr/$T.err
