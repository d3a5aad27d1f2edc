set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -q -x -k "not rank_drop and not two_ranks and not layer" > gpurun_out/t.log 2>&1
timeout -k 10 120 python tools/phase_trace.py > gpurun_out/pt.txt 2>&1
timeout -k 10 240 python bench.py --no-epoch > gpurun_out/b.json 2> gpurun_out/b.err
