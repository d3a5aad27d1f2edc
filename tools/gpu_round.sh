set -e
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/b_default.json 2> gpurun_out/b.err
DNN_FORCE_COLLECTIVES=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29544 timeout -k 10 300 python bench.py --steps 3000 --warmup 300 > gpurun_out/b_forced_epochavg.json 2> gpurun_out/bf.err
