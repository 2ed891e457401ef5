#!/bin/bash
# round 6: embedding gradient one wave per position (k_tr_embed_bwd4, since removed) -- bitwise against the previous
# build (abvar/base.so), training tests, interleaved A/B
set -o pipefail
mkdir -p gpurun_out/eb /tmp/abeb
for dt in bf16 fp32; do
  AA_LIB_PATH=$PWD/abvar/base.so timeout -k 10 120 python -u tools/ab_bits.py dump /tmp/abeb/base_$dt.npz --train $dt > /dev/null 2>> gpurun_out/eb/bits.err || exit 1
  timeout -k 10 120 python -u tools/ab_bits.py dump /tmp/abeb/new_$dt.npz --train $dt > /dev/null 2>> gpurun_out/eb/bits.err || exit 1
  echo "== $dt"; python3 tools/ab_bits.py cmp /tmp/abeb/base_$dt.npz /tmp/abeb/new_$dt.npz | tail -1
done > gpurun_out/eb/bits.txt 2>&1
rm -rf /tmp/abeb; cat gpurun_out/eb/bits.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_configs.py > gpurun_out/eb/pytest.log 2>&1 && echo pytest-ok || exit 1
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then export AA_LIB_PATH=$PWD/abvar/base.so; else unset AA_LIB_PATH; fi
    timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/eb/b_${v}_${rep}.json 2>> gpurun_out/eb/b.err || exit 1
    echo "$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/eb/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
unset AA_LIB_PATH
