# Image staging A/B: engine GPU tests, then the default bench with staging on / off and the
# driver's short run, plus a kernel trace of the staged step.
# usage (repo root, via gpurun): bash tools/gpu_stage.sh [outdir]
set -e
O=gpurun_out/${1:-stage}
mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -v --timeout 300 \
  --timeout-method thread > $O/t.log 2>&1
for k in 1 2; do
  DNN_STAGE_IMAGES=1 timeout -k 10 300 python bench.py > $O/on$k.json 2> $O/on$k.err
  DNN_STAGE_IMAGES=0 timeout -k 10 300 python bench.py > $O/off$k.json 2> $O/off$k.err
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/k20.json 2> $O/k20.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- \
  python3 $R/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
