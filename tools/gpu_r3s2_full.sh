set -e
# whole GPU suite + smoke on the current tree
O=gpurun_out/${1:-r3s2_full}
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/t.log 2>&1
