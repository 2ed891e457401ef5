#!/bin/bash
# A/B of the sequential decode over several (library, flags) configurations, interleaved, two reps.
# usage (GPU box): CONFIGS="tag:lib:flags tag2:lib2:flags2 ..." bash tools/gpu_ab.sh <outdir>
# Prints per config: captions/s, ms per batch and every traced kernel's median (us).
set -u
out=${1:-gpurun_out/ab}
mkdir -p $out
for rep in 1 2; do
  for cfg in $CONFIGS; do
    IFS=: read -r tag lib flags <<< "$cfg"
    AA_LIB_PATH=$PWD/$lib timeout -k 10 150 python bench.py --no-cpu-baseline --no-eval-loop --pipeline-depth 1 --steps 20 \
      --decode-flags ${flags:-0} > $out/ab_${tag}_$rep.json 2> $out/ab_${tag}_$rep.err \
      || { echo "bench failed: $tag"; tail -5 $out/ab_${tag}_$rep.err; exit 1; }
    python3 - $out/ab_${tag}_$rep.json ${tag}_$rep <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = ' '.join(f'{n}={v["median_ms"]*1e3:.2f}' for n, v in d['kernels'].items())
print(sys.argv[2], 'seq', round(d['value']), 'ms', round(d['ms_per_step'], 4), k)
PY
  done
done
