set -e
# DPP cross-lane reductions in both kernels: bf16 phase trace + benches, fp32 bench, whole GPU suite
O=gpurun_out/${1:-r3s2_k}
rm -rf $O; mkdir -p $O
timeout -k 10 120 python tools/phase_trace.py > $O/phase_bf16.txt 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b_k20.json 2> $O/b_k20.err
timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-epoch > $O/b_2k.json 2> $O/b_2k.err
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b_k20b.json 2> $O/b_k20b.err
timeout -k 10 120 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/b32_k20.json 2> $O/b32_k20.err
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/t.log 2>&1
