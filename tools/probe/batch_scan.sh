set -e
for B in 512 1024 2048; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-trace --steps 30 --batch $B --pipeline-depth 1 > gpurun_out/bb.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/bb.json'));print('B', $B, 'seq captions/s', round(d['sequential']['value']), 'ms/batch', round(d['sequential']['ms_per_step'],3))"
done
for D in 2 3 4 6; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-trace --steps 40 --pipeline-depth $D > gpurun_out/bb.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/bb.json'));print('depth', $D, 'pipe captions/s', round(d['value']), 'ms/batch', round(d['ms_per_step'],3))"
done
