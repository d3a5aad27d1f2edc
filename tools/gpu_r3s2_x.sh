set -e
# probe: bench only (20/5 twice, 2000 steps)
O=gpurun_out/${1:-r3s2_x}
rm -rf $O; mkdir -p $O
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-epoch > $O/b_k20.json 2> $O/b_k20.err
timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-epoch > $O/b_2k.json 2> $O/b_2k.err
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-epoch > $O/b_k20b.json 2> $O/b_k20b.err
