set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 300 python tools/phase_trace.py > gpurun_out/phase.txt 2>&1
timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch > gpurun_out/b_default.json 2> gpurun_out/b.err
