#!/bin/bash
# A candidate build against a reference build on one box: the decode parity + pipeline + beam GPU tests
# through the candidate (AA_LIB_PATH), then tools/ab.sh over both.  usage: bash tools/gpu_ab_lib.sh <tag> <ref.so> <cand.so>
set -u
tag=$1; a=$2; b=$3
out=gpurun_out/$tag; mkdir -p $out
AA_LIB_PATH=$PWD/$b timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_beam.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest.log 2>&1
rc=$?; echo "[tests] exit $rc"; tail -4 $out/pytest.log
[ $rc -ne 0 ] && exit $rc
LIBS="$a $b" bash tools/ab.sh > $out/ab.txt 2>&1; rc=$?
cat $out/ab.txt; exit $rc
