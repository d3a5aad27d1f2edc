set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/xg_t.log 2>&1
DNN_FORCE_COLLECTIVES=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29700 timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch > gpurun_out/b_force_xgmi.json 2> gpurun_out/b_force_xgmi.err
DNN_FORCE_COLLECTIVES=1 DNN_ALLREDUCE=rccl MASTER_ADDR=127.0.0.1 MASTER_PORT=29701 timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch > gpurun_out/b_force_rccl.json 2> gpurun_out/b_force_rccl.err
