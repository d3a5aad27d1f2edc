set -e
mkdir -p gpurun_out/xab
export DNN_FORCE_COLLECTIVES=1 MASTER_ADDR=127.0.0.1
for f in 3 0 1 2; do
  DNN_XGMI_FENCES=$f MASTER_PORT=2971$f timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch > gpurun_out/xab/f$f.json 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp
DNN_XGMI_FENCES=3 MASTER_PORT=29720 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/xab/prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
DNN_XGMI_FENCES=0 MASTER_PORT=29721 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/xab/prof0 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
