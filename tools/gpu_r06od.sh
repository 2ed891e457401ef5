#!/bin/bash
# round 6: raw stream handle + on_device (no device switch when current) -- check, GPU tests, training bench
set -o pipefail
mkdir -p gpurun_out/od
timeout -k 10 120 python -u tools/stream_handle_check.py > gpurun_out/od/check.txt 2>&1 && cat gpurun_out/od/check.txt | tail -1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -o cache_dir=/tmp/pc > gpurun_out/od/pytest.log 2>&1 && tail -1 gpurun_out/od/pytest.log || exit 1
timeout -k 10 120 python -u tools/train_host_probe.py > gpurun_out/od/host.txt 2>&1 && grep "per phase" gpurun_out/od/host.txt
timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/od/b.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/od/b.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))"
