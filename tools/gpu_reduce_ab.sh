# A/B of the standalone grad_reduce work-group size (DNN_REDUCE_WAVES = 4, 2, 1 waves per group):
# exactness tests, headline bench and per-kernel stats for each.  usage: bash tools/gpu_reduce_ab.sh
# (the DNN_REDUCE_WAVES knob was reverted after this A/B: profiles/r1_reduce_wg_size_experiment.txt)
set -e
mkdir -p gpurun_out/rab
R=$PWD
for w in 4 2 1; do
  DNN_REDUCE_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
    --timeout 120 --timeout-method thread -k "reduction_is_exact or bitwise or deterministic or track_cpu" \
    > gpurun_out/rab/t_$w.log 2>&1
  DNN_REDUCE_WAVES=$w timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch \
    > gpurun_out/rab/b_$w.json 2> gpurun_out/rab/b_$w.err
done
for w in 4 2 1; do
  DNN_REDUCE_WAVES=$w timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch \
    > gpurun_out/rab/b2_$w.json 2> gpurun_out/rab/b2_$w.err
done
cd /tmp && export TMPDIR=/tmp
for w in 4 1; do
  DNN_REDUCE_WAVES=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rab/prof_$w -o run -- \
    python3 $R/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
done
