# Rank-drop recovery rehearsal on the one-GPU box (ranks share GPU 0, gloo host collectives,
# xGMI exchange between the ranks' IPC regions).  usage (repo root, via gpurun): bash tools/gpu_fault_rehearsal.sh
set -e
O=gpurun_out/fault
mkdir -p $O
for n in 3 4; do
  timeout -k 10 300 python tools/fault_bench.py -n $n --share-gpu --train-samples 6144 --test-samples 1024 --timeout 240 \
    > $O/f$n.json 2> $O/f$n.err
done
