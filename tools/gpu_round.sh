set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_layers_gpu.py -m gpu -q -rA > gpurun_out/tl.log 2>&1
