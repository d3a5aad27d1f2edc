set -e
# end-of-round PMC pass of both fused training kernels (8 SQ counters each, one pass per kernel run)
O=gpurun_out/${1:-r3s2_pmc}
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d $O/pmc_bf16 -- python tools/phase_trace.py > $O/pmc_bf16.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d $O/pmc_fp32 -- python tools/phase_trace_f32.py > $O/pmc_fp32.log 2>&1
