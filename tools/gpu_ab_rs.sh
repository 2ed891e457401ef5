#!/bin/bash
# Fused-rescoring check: the decode parity + pipeline GPU tests, then an interleaved A/B of two builds.
# usage (GPU box): bash tools/gpu_ab_rs.sh <tag> <libA> <libB>
set -u
tag=$1; a=$2; b=$3
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest.log 2>&1
rc=$?; echo "[tests] exit $rc"; tail -5 $out/pytest.log
[ $rc -ne 0 ] && exit $rc
LIBS="$a $b" bash tools/ab.sh > $out/ab.txt 2>&1; rc=$?
cat $out/ab.txt; exit $rc
