#!/bin/bash
# round 6: k_vexact variants A/B: vx0 (one tile per workgroup, 3 per CU), vxp2 (persistent, 2 per CU), this tree (persistent, 3 per CU)
set -o pipefail
mkdir -p gpurun_out/vx2
for rep in 1 2; do
  for v in vx0 vxp2 tree; do
    if [ $v = tree ]; then unset AA_LIB_PATH; else export AA_LIB_PATH=$PWD/abvar/$v.so; fi
    timeout -k 10 200 python -u bench_beam.py --no-cpu-baseline > gpurun_out/vx2/b_${v}_${rep}.json 2>> gpurun_out/vx2/b.err || exit 1
    echo "$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/vx2/b_${v}_${rep}.json'));r=d.get('roofline',{});print(round(d['value']),round(d['ms_per_step'],3), r.get('frac'))")"
  done
done
unset AA_LIB_PATH
