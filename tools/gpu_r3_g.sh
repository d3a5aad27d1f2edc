set -e
# fp32 kernel trace + tests, xGMI exchange tests (bf16 granules included)
O=gpurun_out/r3_g
mkdir -p $O
timeout -k 10 120 python tools/phase_trace_f32.py > $O/phase_f32.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k f32 -x -q --timeout 120 --timeout-method thread > $O/t_f32.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $O/t_xgmi.log 2>&1
