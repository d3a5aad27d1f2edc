set -e
# current tree: fp32 kernel PMC pass (same 8 SQ counters as profiles/r3/fp32/pmc_train_kernel.txt)
# + kernel statistics of both engines over 2000 steps
O=gpurun_out/${1:-r3s2_prof}
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d $O/pmc/p1 -- python tools/phase_trace_f32.py > $O/pmc.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2000 --warmup 200 --no-epoch > $O/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof32 -o run -- python3 bench.py --dtype fp32 --steps 2000 --warmup 200 --no-epoch > $O/prof32.log 2>&1
