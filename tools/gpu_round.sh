set -e
mkdir -p gpurun_out
export DNN_FORCE_COLLECTIVES=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 300 python bench.py --steps 3000 --warmup 300 --no-epoch > gpurun_out/bf.json 2> gpurun_out/bf.err
