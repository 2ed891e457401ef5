#!/bin/bash
# round 6: zero_grad fast paths (Encoder2Decoder, adaptive_amd.optim.Adam) -- tests, interleaved A/B (AA_FAST_ZG=0: torch's)
set -o pipefail
mkdir -p gpurun_out/zg
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_configs.py tests/test_gpu_optim.py > gpurun_out/zg/pytest.log 2>&1 && echo pytest-ok || exit 1
for rep in 1 2 3; do
  for v in 1 0; do
    AA_FAST_ZG=$v timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/zg/b_${v}_${rep}.json 2>> gpurun_out/zg/b.err || exit 1
    echo "fast_zg=$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/zg/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
AA_FAST_ZG=1 timeout -k 10 120 python -u tools/train_host_probe.py > gpurun_out/zg/host1.txt 2>&1 && AA_FAST_ZG=0 timeout -k 10 120 python -u tools/train_host_probe.py > gpurun_out/zg/host0.txt 2>&1 && grep "per phase" gpurun_out/zg/host1.txt gpurun_out/zg/host0.txt
