#!/bin/bash
# round 6: training gradients as views of one allocation -- parity, then interleaved A/B (AA_FLAT_GRADS=0: per-tensor)
set -o pipefail
mkdir -p gpurun_out/z2
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_configs.py tests/test_gpu_optim.py > gpurun_out/z2/pytest.log 2>&1 && echo pytest-ok || exit 1
for rep in 1 2 3; do
  for v in 1 0; do
    AA_FLAT_GRADS=$v timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/z2/b_${v}_${rep}.json 2>> gpurun_out/z2/b.err || exit 1
    echo "flat=$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/z2/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
timeout -k 10 120 python -u tools/train_host_probe.py > gpurun_out/z2/host.txt 2>&1 && echo host-ok
