set -e
for extra in "" "--pool-streams"; do
for D in 2 3 4 6; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-trace --steps 40 --pipeline-depth $D $extra > gpurun_out/bb.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/bb.json'));print('depth', $D, '$extra', 'pipe', round(d['value']), 'seq', round(d['sequential']['value']))"
done; done
