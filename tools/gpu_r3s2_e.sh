set -e
# fp32 kernel: numerics, phase timeline, bench (20/5 + 2000 steps)
O=gpurun_out/${1:-r3s2_e}
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k f32 -x -v --timeout 120 --timeout-method thread > $O/t_f32.log 2>&1
timeout -k 10 120 python tools/phase_trace_f32.py > $O/phase_f32.txt 2>&1
timeout -k 10 120 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/b_f32_k20.json 2> $O/b_f32_k20.err
timeout -k 10 120 python bench.py --dtype fp32 --steps 2000 --warmup 200 --no-epoch > $O/b_f32_2k.json 2> $O/b_f32_2k.err
