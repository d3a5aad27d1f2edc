# XCD-aware sample placement A/B on the headline step + phase trace; rank-drop test with the
# map off (flakiness baseline).  usage (from the repo root, via gpurun): bash tools/gpu_xcd_ab.sh
set -e
mkdir -p gpurun_out/xcd
rm -f gpurun_out/xcd/ab_*.jsonl
timeout -k 10 300 python tools/phase_trace.py > gpurun_out/xcd/phase.txt 2>&1
for m in 1 0 1 0 1 0; do
  DNN_XCD_MAP=$m timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch \
    >> gpurun_out/xcd/ab_map$m.jsonl 2>> gpurun_out/xcd/ab.err
done
: > gpurun_out/xcd/drop.txt
for i in 1 2 3; do
  if DNN_XCD_MAP=0 timeout -k 10 200 python -u -m pytest "tests/test_engine_gpu.py::test_rank_drop_recovery_on_gpu_engine[step-allreduce]" \
      -x -q --timeout 180 --timeout-method thread > gpurun_out/xcd/drop$i.log 2>&1; then
    echo "map0 run $i pass" >> gpurun_out/xcd/drop.txt
  else
    echo "map0 run $i FAIL" >> gpurun_out/xcd/drop.txt
  fi
done
