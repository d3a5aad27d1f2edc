# A/B of the next-step L2 image warm-up in grad_reduce (DNN_PREFETCH=1 default, 0 = off):
# exactness tests, headline bench (interleaved, twice each) and kernel stats.
# usage (repo root, via gpurun): bash tools/gpu_prefetch_ab.sh
# (the DNN_PREFETCH knob was reverted after this A/B: profiles/r1_prefetch_experiment.txt)
set -e
mkdir -p gpurun_out/pf
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pf/t.log 2>&1
for i in 1 2; do
  for p in 1 0; do
    DNN_PREFETCH=$p timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch \
      > gpurun_out/pf/b${i}_$p.json 2> gpurun_out/pf/b${i}_$p.err
  done
done
timeout -k 10 300 python tools/phase_trace.py > gpurun_out/pf/phase_1.txt 2>&1
DNN_PREFETCH=0 timeout -k 10 300 python tools/phase_trace.py > gpurun_out/pf/phase_0.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pf/prof_1 -o run -- \
  python3 $R/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
