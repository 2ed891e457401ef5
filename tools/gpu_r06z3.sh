#!/bin/bash
# round 6: k_bgemm split target (AA_BG_WG workgroups) against the training step
set -o pipefail
mkdir -p gpurun_out/z3
for rep in 1 2; do
  for v in 256 128 192 64; do
    AA_BG_WG=$v timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/z3/b_${v}_${rep}.json 2>> gpurun_out/z3/b.err || exit 1
    echo "bg_wg=$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/z3/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
