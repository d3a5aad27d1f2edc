set -e
mkdir -p gpurun_out/ep
for v in sync pinmain async sync pinmain; do
DNN_EB=$v timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch > gpurun_out/ep/full_$v.json 2>/dev/null
DNN_EB=$v timeout -k 10 300 python bench.py --steps 5000 --warmup 500 --no-epoch --train-samples 6400 > gpurun_out/ep/short_$v.json 2>/dev/null
python -c "import json;print('$v', json.load(open('gpurun_out/ep/full_$v.json'))['ms_per_step'], json.load(open('gpurun_out/ep/short_$v.json'))['ms_per_step'])" >> gpurun_out/ep/summary.txt
done
