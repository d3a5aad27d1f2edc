# Kernel trace + PMC counters of the conv kernels on the cifar-vgg layer shapes.
# usage (from the repo root, via gpurun): bash tools/gpu_pmc_conv.sh
set -e
mkdir -p gpurun_out/pmc
R=$PWD
: > gpurun_out/pmc/t.txt
for cfg in "fwd 64 32 32 32 3 1" "fwd 64 64 16 64 3 1" "dgrad 64 32 32 32 3 1" "wgrad 64 32 32 32 3 1" "wgrad 64 64 16 64 3 1"; do
  timeout -k 10 120 python tools/conv_micro.py $cfg 1 200 >> gpurun_out/pmc/t.txt 2>&1
done
cd /tmp && export TMPDIR=/tmp
for cfg in "fwd 64 32 32 32 3 1" "fwd 64 64 16 64 3 1"; do set -- $cfg; tag=$1_$3_$4
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc/p1_$tag -o run -- python3 $R/tools/conv_micro.py $cfg 1 20 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmc/p2_$tag -o run -- python3 $R/tools/conv_micro.py $cfg 1 20 > /dev/null 2>&1
done
