set -e
O=gpurun_out/r3_b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
DNN_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29701 bench.py --gpus 2 --steps 200 --warmup 20 > $O/bench2.json 2> $O/bench2.err
timeout -k 10 400 python -u tools/fault_bench.py -n 4 --share-gpu --epochs 3 --train-samples 20000 --test-samples 2000 --log $O/fault4.log > $O/fault4.json 2> $O/fault4.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 2000 --warmup 200 --no-epoch > $O/prof.log 2>&1
