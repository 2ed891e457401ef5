#!/bin/bash
# Bench several decode configurations back to back on one GPU box (A/B of options, not builds).
# usage: bash tools/variants.sh "<label>:<bench.py args>" ...   e.g. "fused:" "split:--split-lstm --no-graph"
# Prints per variant: sequential / pipelined captions/s and the traced per-kernel averages (us).
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  label=${spec%%:*}
  args=${spec#*:}
  timeout -k 10 180 python bench.py --no-cpu-baseline --steps ${STEPS:-30} $args > gpurun_out/var_$label.json 2> gpurun_out/var_$label.err \
    || { echo "variant $label failed"; tail -5 gpurun_out/var_$label.err; exit 1; }
  echo "$label $(python -c "
import json;d=json.load(open('gpurun_out/var_$label.json'))
k=' '.join(f'{n}={v[\"avg_ms\"]*1e3:.2f}' for n,v in d['kernels'].items())
print('seq', round(d['value']), 'pipe', round(d['pipelined']['value']), 'ms', round(d['ms_per_step'],4), k)")"
done
