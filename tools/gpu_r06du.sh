#!/bin/bash
# round 6: dU's own k_bgemm split target (AA_BG_WG_DU, a switch since removed) against the default 256
set -o pipefail
mkdir -p gpurun_out/du
for rep in 1 2; do
  for v in 0 512 1024 128; do
    AA_BG_WG_DU=$v timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/du/b_${v}_${rep}.json 2>> gpurun_out/du/b.err || exit 1
    echo "du_wg=$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/du/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
