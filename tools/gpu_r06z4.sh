#!/bin/bash
# round 6: k_tgemm deep-split target (AA_TG_DEEP_WG) with k_bgemm at 256 workgroups
set -o pipefail
mkdir -p gpurun_out/z4
for rep in 1 2; do
  for v in 1024 512 256; do
    AA_TG_DEEP_WG=$v timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/z4/b_${v}_${rep}.json 2>> gpurun_out/z4/b.err || exit 1
    echo "deep_wg=$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/z4/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
