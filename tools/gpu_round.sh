set -e
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_engine_gpu.py -m gpu -q -k "rank_drop" -rA > gpurun_out/t3.log 2>&1
