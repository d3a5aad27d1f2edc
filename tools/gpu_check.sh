set -e
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/b_default.json 2> gpurun_out/b.err
