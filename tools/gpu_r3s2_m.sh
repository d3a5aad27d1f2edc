set -e
# grad_reduce fc tiles with two accumulator chains: reduction tests, per-block trace, bench
O=gpurun_out/${1:-r3s2_m}
rm -rf $O; mkdir -p $O
timeout -k 10 120 python tools/reduce_trace.py > $O/reduce_trace.txt 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b_k20.json 2> $O/b_k20.err
timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-epoch > $O/b_2k.json 2> $O/b_2k.err
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b_k20b.json 2> $O/b_k20b.err
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_xgmi_gpu.py tests/test_parity_gpu.py -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1
