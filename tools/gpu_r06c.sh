#!/bin/bash
# Round 6: per-workgroup phase marks of the fused LSTM + attention launch (tools/ktrace_at.py) with the
# instrumented builds (abvar/at_ts.so: V prefetched under the GEMM; abvar/at_ts_nopf.so: V loaded once
# the block is ready).
set -u
out=gpurun_out/r06c
mkdir -p $out
for v in ${VARIANTS:-at_ts at_ts_nopf}; do
  [ -f abvar/$v.so ] || continue
  AA_LIB_PATH=$PWD/abvar/$v.so timeout -k 10 120 python tools/ktrace_at.py > $out/ktrace_$v.txt 2>&1
  rc=$?; echo "[$v] exit $rc"; cat $out/ktrace_$v.txt | tail -25
  [ $rc -eq 0 ] || exit $rc
done
