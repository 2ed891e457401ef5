set -e
cd /root/repo
for rep in 1 2; do
for opt in "" "--screen64"; do
for d in 2 4; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-trace --steps 100 --pipeline-depth $d $opt > gpurun_out/co.json
  echo "rep$rep [$opt] depth $d $(python -c "import json;d=json.load(open('gpurun_out/co.json'));print(round(d['value']), round(d['ms_per_step'],4), round(d['sequential']['value']))")"
done
done
done
