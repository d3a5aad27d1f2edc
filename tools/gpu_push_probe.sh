# Exchange-form probe on the one-GPU box: N ranks time-sharing the GPU train 4 epochs each
# (tools/push_probe.py, 5 s wait bound).  usage (repo root, via gpurun): bash tools/gpu_push_probe.sh
set -e
O=gpurun_out/pprobe
mkdir -p $O
for cfg in "rsag 0 4" "rsag 0 4" "rsag 0 4" "push 0 2" "pull 0 4"; do set -- $cfg
  DNN_XGMI_EXCHANGE=$1 DNN_XGMI_AR_PUSH=$2 DNN_XGMI_TIMEOUT_S=5 DNN_BACKEND=gloo OMP_NUM_THREADS=2 \
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $3 --master-addr 127.0.0.1 \
    --master-port 29741 tools/push_probe.py >> $O/p_$1_$3.out 2>> $O/p_$1_$3.err || echo "rc=$? $cfg" >> $O/rc.txt
done
