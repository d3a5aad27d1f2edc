set -e
mkdir -p gpurun_out/fab
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fab/t.log 2>&1
timeout -k 10 300 python tools/phase_trace.py > gpurun_out/fab/phase.txt 2>&1
for i in 1 2; do timeout -k 10 200 python bench.py --steps 5000 --warmup 500 --no-epoch > gpurun_out/fab/b5000_$i.json 2> gpurun_out/fab/b5000_$i.err; done
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/fab/b20_$i.json 2> gpurun_out/fab/b20_$i.err; done
