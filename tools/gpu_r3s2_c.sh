set -e
O=gpurun_out/${1:-r3s2_c}
rm -rf $O; mkdir -p $O
timeout -k 10 120 python tools/phase_trace_f32.py > $O/phase_f32.txt 2>&1
