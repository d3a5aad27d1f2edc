# Kernel-boundary cost under HIP runtime knobs: the launch probe, then the layer-engine lenet
# bench, once per setting.  usage (repo root, via gpurun): bash tools/gpu_launch_probe.sh [outdir]
set -e
O=gpurun_out/${1:-lprobe}
mkdir -p $O
run() {  # label, env assignments...
  local label=$1; shift
  env "$@" timeout -k 10 120 python tools/launch_probe.py $label >> $O/probe.jsonl 2>> $O/probe.err
  env "$@" timeout -k 10 200 python bench.py --model lenet --dtype fp32 --engine layers --steps 300 --warmup 30 \
    --no-epoch > $O/b_lenet_$label.json 2> $O/b_lenet_$label.err
  echo "$label done"
}
run default
run devkernarg HIP_FORCE_DEV_KERNARG=1
run nodevkernarg HIP_FORCE_DEV_KERNARG=0
run nopktcap DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
