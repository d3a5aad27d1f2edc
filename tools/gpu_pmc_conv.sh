set -e
mkdir -p gpurun_out/pmc
R=$PWD
timeout -k 10 120 python tools/conv_micro.py 64 32 16 64 3 1 1 200 > gpurun_out/pmc/t.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc/kt -o run -- python3 $R/tools/conv_micro.py 64 32 16 64 3 1 1 50 > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc/p1 -o run -- python3 $R/tools/conv_micro.py 64 32 16 64 3 1 1 20 > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d $R/gpurun_out/pmc/p2 -o run -- python3 $R/tools/conv_micro.py 64 32 16 64 3 1 1 20 > /dev/null 2>&1
