# PMC counters of the layer-engine kernels (cifar-vgg bf16 step), two passes within the per-block
# counter limits.  usage (repo root, via gpurun): bash tools/gpu_pmc_layers.sh [outdir]
set -e
O=gpurun_out/${1:-pmcl}
mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  -d $R/$O/pmc1 -o run -- python3 $R/bench.py --model cifar-vgg --dtype bf16 --engine layers --steps 8 --warmup 2 \
  --no-epoch --no-graphs > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  -d $R/$O/pmc2 -o run -- python3 $R/bench.py --model cifar-vgg --dtype bf16 --engine layers --steps 8 --warmup 2 \
  --no-epoch --no-graphs > /dev/null 2>&1
