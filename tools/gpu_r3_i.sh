set -e
# early-MLP overlap: bitwise tests (1 rank, 2 ranks), then bench A/B (serial vs early) at k20 and 2000 steps
O=gpurun_out/r3_i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k early_mlp -x -v --timeout 200 --timeout-method thread > $O/t_early.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -k early_mlp -x -v --timeout 250 --timeout-method thread > $O/t_early_xgmi.log 2>&1
for m in off mlp full; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --early-mlp $m > $O/b_k20_$m.json 2> $O/b_k20_$m.err
  timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-epoch --early-mlp $m > $O/b_2k_$m.json 2> $O/b_2k_$m.err
done
