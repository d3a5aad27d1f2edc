set -e
# fp32 kernel under rocprofv3 --kernel-trace vs plain: is the 2x a profiler effect?
O=gpurun_out/${1:-r3s2_d}
rm -rf $O; mkdir -p $O
timeout -k 10 120 python bench.py --dtype fp32 --steps 2000 --warmup 200 --no-epoch > $O/b32_plain.json 2> $O/b32_plain.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt32 -o run -- python3 bench.py --dtype fp32 --steps 2000 --warmup 200 --no-epoch > $O/b32_kt.json 2> $O/b32_kt.err
timeout -k 10 120 python bench.py --dtype fp32 --steps 2000 --warmup 200 --no-epoch > $O/b32_plain2.json 2> $O/b32_plain2.err
