set -e
mkdir -p gpurun_out
timeout -k 10 120 python tools/reduce_trace.py > gpurun_out/rt.txt 2>&1
