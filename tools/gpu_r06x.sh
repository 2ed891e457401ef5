#!/bin/bash
# round 6: bitwise check of the transposed-weight backward against the previous build (abvar/base.so)
set -o pipefail
mkdir -p gpurun_out/x /tmp/abx
for dt in bf16 fp32; do
  AA_LIB_PATH=$PWD/abvar/base.so timeout -k 10 120 python -u tools/ab_bits.py dump /tmp/abx/base_$dt.npz --train $dt > /dev/null 2>> gpurun_out/x/bits.err || exit 1
  timeout -k 10 120 python -u tools/ab_bits.py dump /tmp/abx/new_$dt.npz --train $dt > /dev/null 2>> gpurun_out/x/bits.err || exit 1
  AA_TG128=1 timeout -k 10 120 python -u tools/ab_bits.py dump /tmp/abx/new1_$dt.npz --train $dt > /dev/null 2>> gpurun_out/x/bits.err || exit 1
  echo "== $dt: previous build vs this build (default)"; python3 tools/ab_bits.py cmp /tmp/abx/base_$dt.npz /tmp/abx/new_$dt.npz
  echo "== $dt: previous build vs this build with AA_TG128=1"; python3 tools/ab_bits.py cmp /tmp/abx/base_$dt.npz /tmp/abx/new1_$dt.npz
done > gpurun_out/x/bits.txt 2>&1
rm -rf /tmp/abx
echo bits-done
