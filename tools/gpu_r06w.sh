#!/bin/bash
# round 6: transposed weight copies for the backward + k_tgemm128 on the deep weight gradients --
# bitwise check against the previous build (abvar/base.so), parity tests, interleaved A/B
set -o pipefail
mkdir -p gpurun_out/w
for dt in bf16 fp32; do
  AA_LIB_PATH=$PWD/abvar/base.so timeout -k 10 120 python -u tools/ab_bits.py dump gpurun_out/w/base_$dt.npz --train $dt > /dev/null 2>> gpurun_out/w/bits.err || exit 1
  AA_TG128=0 timeout -k 10 120 python -u tools/ab_bits.py dump gpurun_out/w/new0_$dt.npz --train $dt > /dev/null 2>> gpurun_out/w/bits.err || exit 1
  AA_TG128=1 timeout -k 10 120 python -u tools/ab_bits.py dump gpurun_out/w/new1_$dt.npz --train $dt > /dev/null 2>> gpurun_out/w/bits.err || exit 1
  echo "== $dt: base vs new (64 x 64 engine only)"; python3 tools/ab_bits.py cmp gpurun_out/w/base_$dt.npz gpurun_out/w/new0_$dt.npz
  echo "== $dt: base vs new (default)"; python3 tools/ab_bits.py cmp gpurun_out/w/base_$dt.npz gpurun_out/w/new1_$dt.npz
done > gpurun_out/w/bits.txt 2>&1
echo bits-done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_configs.py tests/test_gpu_optim.py > gpurun_out/w/pytest.log 2>&1 && echo pytest-ok || exit 1
for rep in 1 2; do
  for v in new1 new0 base; do
    case $v in new1) env="AA_TG128=1";; new0) env="AA_TG128=0";; base) env="AA_LIB_PATH=$PWD/abvar/base.so";; esac
    env $env timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/w/b_${v}_${rep}.json 2>> gpurun_out/w/b.err || exit 1
    echo "$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/w/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
