#!/bin/bash
# Round 6: first run of the fused LSTM + attention launch (k_lstm<512, .., AT>): the parity file
# (fused == split attention == the fallbacks, bit for bit; goldens), then an A/B of the sequential
# decode: fused (default) / split attention (flag 4096) / the late-operand build (abvar/at_late1.so).
set -u
out=gpurun_out/r06b
mkdir -p $out
step() {
  local name=$1; shift
  "$@"; local rc=$?
  echo "[$name] exit $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] crashed or timed out: stopping"; exit $rc; fi
}
step parity timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest_parity.log 2>&1
grep -E "PASSED|FAILED|ERROR|passed|failed" $out/pytest_parity.log | tail -40
grep -q " passed" $out/pytest_parity.log && ! grep -q "FAILED\|ERROR" $out/pytest_parity.log || { echo "parity not green: stopping"; exit 1; }
run() {  # tag, lib, extra args
  local tag=$1 lib=$2; shift 2
  AA_LIB_PATH=$PWD/$lib timeout -k 10 150 python bench.py --no-cpu-baseline --no-eval-loop --pipeline-depth 1 --steps 20 "$@" \
    > $out/ab_$tag.json 2> $out/ab_$tag.err || { echo "bench failed: $tag"; tail -5 $out/ab_$tag.err; exit 1; }
  python3 - $out/ab_$tag.json $tag <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = ' '.join(f'{n}={v["median_ms"]*1e3:.2f}' for n, v in d['kernels'].items() if n in ('k_lstm(step0)', 'k_lstm', 'k_atten', 'k_vscreen', 'k_vrescore', 'k_enc_v4'))
print(sys.argv[2], 'seq', round(d['value']), 'ms', round(d['ms_per_step'], 4), k)
PY
}
for rep in 1 2; do
  run fused$rep adaptive_amd/libadaptive_amd.so
  run split$rep adaptive_amd/libadaptive_amd.so --decode-flags 4096
  run late1_$rep abvar/at_late1.so
done
