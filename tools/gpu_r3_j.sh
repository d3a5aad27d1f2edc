set -e
# kernel timeline of the early-MLP (in-launch) step vs the serial step (rocprofv3 kernel trace)
O=gpurun_out/r3_j
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in on off; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$m -- python3 bench.py --steps 300 --warmup 50 --no-epoch --early-mlp $m > $O/b_$m.json 2> $O/b_$m.err
done
