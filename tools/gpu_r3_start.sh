set -e
O=gpurun_out/r3_a
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b_k20.json 2> $O/b_k20.err
timeout -k 10 300 python bench.py > $O/b_default.json 2> $O/b_default.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 2000 --warmup 200 --no-epoch > $O/prof.log 2>&1
