# Repeat the GPU rank-drop recovery test (logic divergence hunt, not a GPU fault): N runs.
set -e
mkdir -p gpurun_out/dd
: > gpurun_out/dd/summary.txt
for i in 1 2 3; do
  if timeout -k 10 200 python -u -m pytest "tests/test_engine_gpu.py::test_rank_drop_recovery_on_gpu_engine[step-allreduce]" \
      -x -q --timeout 180 --timeout-method thread > gpurun_out/dd/run$i.log 2>&1; then
    echo "run $i pass" >> gpurun_out/dd/summary.txt
  else
    echo "run $i FAIL" >> gpurun_out/dd/summary.txt
  fi
done
