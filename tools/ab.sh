#!/bin/bash
# A/B timing of several builds of libadaptive_amd.so in one GPU session (interleaved, 2 rounds).
# usage (GPU box): LIBS="abvar/a.so abvar/b.so" bash tools/ab.sh [extra bench.py args]
# Prints per build: sequential (and pipelined) captions/s, ms per batch, and the traced per-kernel
# medians (us, dispatch timestamps).
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in $LIBS; do
    AA_LIB_PATH=$PWD/$lib timeout -k 10 150 python bench.py --no-cpu-baseline "$@" \
      > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed for $lib"; tail -5 gpurun_out/ab.err; exit 1; }
    echo "rep$rep $(basename $lib) $(python -c "
import json;d=json.load(open('gpurun_out/ab.json'))
k=' '.join(f'{n}={v.get(\"median_ms\", v[\"avg_ms\"])*1e3:.2f}' for n,v in d['kernels'].items() if n in ('k_lstm','k_atten','k_vscreen','k_vrescore','k_enc_v4'))
print('seq', round(d['value']), 'pipe', round(d['pipelined']['value']), 'ms', round(d['ms_per_step'],4), k)")"
  done
done
