set -e
# end-of-session checkpoint on the committed tree: smoke, the whole GPU suite, driver-shaped and
# long-window bench (bf16 + fp32), kernel statistics of both engines
O=gpurun_out/${1:-r3s2_final}
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b_k20.json 2> $O/b_k20.err
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b_k20b.json 2> $O/b_k20b.err
timeout -k 10 300 python bench.py > $O/b_default.json 2> $O/b_default.err
timeout -k 10 120 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/b32_k20.json 2> $O/b32_k20.err
timeout -k 10 300 python bench.py --dtype fp32 > $O/b32_default.json 2> $O/b32_default.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2000 --warmup 200 --no-epoch > $O/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof32 -o run -- python3 bench.py --dtype fp32 --steps 2000 --warmup 200 --no-epoch > $O/prof32.log 2>&1
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/t.log 2>&1
