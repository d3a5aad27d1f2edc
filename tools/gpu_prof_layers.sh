set -e
mkdir -p gpurun_out/pl
cd /tmp && export TMPDIR=/tmp
for m in "cifar-vgg bf16" "lenet-bn fp32"; do set -- $m
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pl/p_$1_$2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model $1 --dtype $2 --engine layers --steps 200 --warmup 20 --no-epoch > /dev/null 2>&1
done
