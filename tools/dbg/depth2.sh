set -e
cd /root/repo
for rep in 1 2; do
for d in 3 4 6 8; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-trace --steps 100 --pipeline-depth $d > gpurun_out/dep.json
  echo "rep$rep depth $d $(python -c "import json;d=json.load(open('gpurun_out/dep.json'));print(round(d['value']), round(d['ms_per_step'],4), round(d['sequential']['value']))")"
done
done
