set -e
O=gpurun_out/r3_h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k f32 -x -q --timeout 120 --timeout-method thread > $O/t_f32.log 2>&1
timeout -k 10 120 python tools/phase_trace_f32.py > $O/phase.txt 2>&1
timeout -k 10 120 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/b_f32_k20.json 2> $O/b_f32_k20.err
