# One-launch xGMI exchange (grad_reduce does reduce + all-reduce + SGD) vs the two-launch
# path: GPU tests of the xGMI / engine paths, then forced 1-rank step timings (the collective
# path runs with a real group of one), fences 3 (multi-GPU default) and 0, plus a kernel trace.
# usage (repo root, via gpurun): bash tools/gpu_onelaunch.sh [outdir]
set -e
O=gpurun_out/${1:-onelaunch}
mkdir -p $O
R=$PWD
export DNN_DEBUG_XGMI=1
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 \
  --timeout-method thread > $O/t.log 2>&1
export DNN_FORCE_COLLECTIVES=1 MASTER_ADDR=127.0.0.1
for one in 1 0; do
  for f in 3 0; do
    DNN_XGMI_ONE_LAUNCH=$one DNN_XGMI_FENCES=$f MASTER_PORT=297$one$f timeout -k 10 300 \
      python bench.py --steps 5000 --warmup 500 --no-epoch > $O/one${one}_f$f.json 2> $O/one${one}_f$f.err
  done
done
unset DNN_FORCE_COLLECTIVES
timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch > $O/local.json 2> $O/local.err
cd /tmp && export TMPDIR=/tmp
DNN_FORCE_COLLECTIVES=1 DNN_XGMI_FENCES=3 MASTER_PORT=29740 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d $R/$O/prof1 -o run -- python3 $R/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
