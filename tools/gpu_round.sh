set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -m gpu -q -k "two_ranks" -rA > gpurun_out/t2.log 2>&1
