#!/bin/bash
# Round 6: the 8-wave vocab screen (k_vscreen8).  Parity file first, then an A/B of the sequential
# decode: default (k_vscreen8) / AA_DECODE_SCREEN4 (k_vscreen2), same library, two reps.
set -u
out=gpurun_out/r06e
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest_parity.log 2>&1
rc=$?; echo "[parity] exit $rc"; tail -4 $out/pytest_parity.log
[ $rc -eq 0 ] || exit $rc
run() {  # tag, lib, extra args
  local tag=$1 lib=$2; shift 2
  AA_LIB_PATH=$PWD/$lib timeout -k 10 150 python bench.py --no-cpu-baseline --no-eval-loop --pipeline-depth 1 --steps 20 "$@" \
    > $out/ab_$tag.json 2> $out/ab_$tag.err || { echo "bench failed: $tag"; tail -5 $out/ab_$tag.err; exit 1; }
  python3 - $out/ab_$tag.json $tag <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = ' '.join(f'{n}={v["median_ms"]*1e3:.2f}' for n, v in d['kernels'].items())
print(sys.argv[2], 'seq', round(d['value']), 'ms', round(d['ms_per_step'], 4), k)
PY
}
for rep in 1 2; do
  run s8_$rep adaptive_amd/libadaptive_amd.so
  run s4_$rep adaptive_amd/libadaptive_amd.so --decode-flags 4096
done
