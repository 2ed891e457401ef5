#!/bin/bash
# round 6: k_bgemm split to ~256 workgroups -- parity and the training bench (interleaved with the old 1024)
set -o pipefail
mkdir -p gpurun_out/z5
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_configs.py tests/test_gpu_optim.py > gpurun_out/z5/pytest.log 2>&1 && echo pytest-ok || exit 1
for rep in 1 2 3; do
  for v in 256 1024; do
    AA_BG_WG=$v timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/z5/b_${v}_${rep}.json 2>> gpurun_out/z5/b.err || exit 1
    echo "bg_wg=$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/z5/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
timeout -k 10 120 python -u bench_train.py > gpurun_out/z5/bench_train.json 2>> gpurun_out/z5/b.err && echo bench-ok
