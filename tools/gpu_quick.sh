# Quick health check on one MI355X: GPU tests, smoke(), default bench, kernel stats of the
# headline step.  usage (repo root, via gpurun): bash tools/gpu_quick.sh [outdir]
set -e
O=gpurun_out/${1:-quick}
mkdir -p $O
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- \
  python3 $R/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
