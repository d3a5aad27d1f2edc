# One-launch xGMI exchange (grad_reduce does reduce + all-reduce + SGD) vs the two-launch
# path: GPU tests of the xGMI / engine paths, then forced 1-rank step timings (the collective
# path runs with a real group of one) and a kernel trace of the one-launch step.
# usage (repo root, via gpurun): [SKIP_TESTS=1] bash tools/gpu_onelaunch.sh [outdir]
set -e
O=gpurun_out/${1:-onelaunch}
mkdir -p $O
R=$PWD
export DNN_DEBUG_XGMI=1
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 \
  --timeout-method thread > $O/t.log 2>&1
export DNN_FORCE_COLLECTIVES=1 MASTER_ADDR=127.0.0.1
for one in 1 0; do
  DNN_XGMI_ONE_LAUNCH=$one MASTER_PORT=2971$one timeout -k 10 300 \
    python bench.py --steps 5000 --warmup 500 --no-epoch > $O/one$one.json 2> $O/one$one.err
done
unset DNN_FORCE_COLLECTIVES
timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch > $O/local.json 2> $O/local.err
cd /tmp && export TMPDIR=/tmp
DNN_FORCE_COLLECTIVES=1 MASTER_PORT=29740 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d $R/$O/prof1 -o run -- python3 $R/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
