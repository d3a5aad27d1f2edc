set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/b_default.json 2> gpurun_out/b.err
