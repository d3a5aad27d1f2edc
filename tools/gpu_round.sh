set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -q -x > gpurun_out/t.log 2>&1
timeout -k 10 120 python tools/reduce_trace.py > gpurun_out/rt.txt 2>&1
timeout -k 10 240 python bench.py --no-epoch > gpurun_out/b.json 2> gpurun_out/b.err
