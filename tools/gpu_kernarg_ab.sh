# Driver-shaped bench (K=20, W=5) with kernel arguments in device memory vs the default, 3 runs
# each, plus the 5000-step steady state.  usage (repo root, via gpurun): bash tools/gpu_kernarg_ab.sh [outdir]
set -e
O=gpurun_out/${1:-kab}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/def_$i.json 2> $O/def_$i.err
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/dev_$i.json 2> $O/dev_$i.err
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/host_$i.json 2> $O/host_$i.err
done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --diag-windows 3 > $O/dev_diag.json 2> $O/dev_diag.err
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --diag-windows 3 > $O/def_diag.json 2> $O/def_diag.err
