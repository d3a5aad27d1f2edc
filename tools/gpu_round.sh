set -e
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > gpurun_out/t.log 2>&1
