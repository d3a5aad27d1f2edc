set -e
# fp32 kernel: tests, phase timeline, bench, and one PMC pass (LDS / VALU issue picture)
O=gpurun_out/r3_e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k f32 -x -q --timeout 120 --timeout-method thread > $O/t_f32.log 2>&1
timeout -k 10 120 python tools/phase_trace_f32.py > $O/phase_f32.txt 2>&1
timeout -k 10 120 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/b_f32_k20.json 2> $O/b_f32_k20.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d $O/pmc -- python tools/phase_trace_f32.py > $O/pmc.log 2>&1
