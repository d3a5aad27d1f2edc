set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/b_def.json 2> gpurun_out/b_def.err
timeout -k 10 240 python bench.py --in-launch-reduce --no-epoch > gpurun_out/b_inl.json 2> gpurun_out/b_inl.err
(cd _ab_head && timeout -k 10 240 python bench.py --steps 5000 --warmup 500 --no-epoch > ../gpurun_out/b_head.json 2> ../gpurun_out/b_head.err)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/p_def -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2000 --warmup 200 --no-epoch > $GRAFT_REPO_ROOT/gpurun_out/p_def.log 2>&1
