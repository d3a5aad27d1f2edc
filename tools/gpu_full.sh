# Round-end rehearsal on one MI355X: every GPU test, smoke(), the default bench line.
# usage (from the repo root, via gpurun): bash tools/gpu_full.sh
set -e
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/full/t.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err
