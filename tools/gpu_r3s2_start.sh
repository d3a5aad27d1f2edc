set -e
# session-2 start: the restored tree still builds-and-runs (driver-shaped bf16 + fp32 bench)
O=gpurun_out/r3s2_start
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b_k20.json 2> $O/b_k20.err
timeout -k 10 120 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/b_f32_k20.json 2> $O/b_f32_k20.err
timeout -k 10 300 python bench.py > $O/b_default.json 2> $O/b_default.err
