#!/bin/bash
# A/B of environment settings against one build, interleaved over 2 rounds (GPU box).
# usage: LIB=tools/_build/x.so bash tools/ab_env.sh "<label>:<ENV=val ...>:<bench.py args>" ...
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    IFS=: read -r label envs args <<< "$spec"
    env ${LIB:+AA_LIB_PATH=$PWD/$LIB} $envs timeout -k 10 150 python bench.py --no-cpu-baseline --steps ${STEPS:-30} $args \
      > gpurun_out/abe.json 2> gpurun_out/abe.err || { echo "bench failed for $label"; tail -5 gpurun_out/abe.err; exit 1; }
    echo "rep$rep $label $(python -c "
import json;d=json.load(open('gpurun_out/abe.json'))
k=' '.join(f'{n}={v[\"avg_ms\"]*1e3:.2f}' for n,v in d['kernels'].items() if n in ('k_lstm','k_atten','k_vscreen','k_vrescore','k_enc_v4'))
print('seq', round(d['value']), 'pipe', round(d['pipelined']['value']), 'ms', round(d['ms_per_step'],4), k)")"
  done
done
