# Round-end evidence on one MI355X: all GPU tests, smoke(), default bench (with epoch time),
# rocprofv3 kernel stats of the headline step, PMC counters of the fused kernel, and the
# layer-engine bench lines.  usage (from the repo root, via gpurun): bash tools/gpu_final.sh
set -e
mkdir -p gpurun_out/final
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/final/t.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench_k20.json 2> gpurun_out/final/bench_k20.err
for m in "cifar-vgg bf16" "cifar-vgg fp32" "lenet-bn fp32" "lenet fp32"; do set -- $m
  timeout -k 10 300 python bench.py --model $1 --dtype $2 --engine layers --steps 300 --warmup 30 --no-epoch \
    > gpurun_out/final/b_$1_$2.json 2> gpurun_out/final/b_$1_$2.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final/prof -o run -- \
  python3 $R/bench.py --steps 2000 --warmup 200 --no-epoch > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  -d $R/gpurun_out/final/pmc1 -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-epoch --no-graphs > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  -d $R/gpurun_out/final/pmc2 -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-epoch --no-graphs > /dev/null 2>&1
