set -e
O=gpurun_out/r3_c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k f32 -x -v --timeout 120 --timeout-method thread > $O/t_f32.log 2>&1
timeout -k 10 120 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/b_f32_k20.json 2> $O/b_f32_k20.err
timeout -k 10 300 python bench.py --dtype fp32 --steps 2000 --warmup 200 > $O/b_f32.json 2> $O/b_f32.err
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -v -s --timeout 400 --timeout-method thread > $O/t_parity.log 2>&1
timeout -k 10 400 python -u tools/fault_bench.py -n 4 --share-gpu --epochs 3 --train-samples 20000 --test-samples 2000 --log $O/fault4.log > $O/fault4.json 2> $O/fault4.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --dtype fp32 --steps 1000 --warmup 100 --no-epoch > $O/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof16 -o run -- python bench.py --steps 2000 --warmup 200 --no-epoch > $O/prof16.log 2>&1
