#!/bin/bash
# round 6: training step time against batch size (is the step bound by GPU work or by launches?)
set -o pipefail
mkdir -p gpurun_out/y
for b in 32 64 128 256; do
  timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 --batch $b > gpurun_out/y/b$b.json 2>> gpurun_out/y/err || exit 1
  echo "B=$b $(python3 -c "import json;d=json.load(open('gpurun_out/y/b$b.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
done
