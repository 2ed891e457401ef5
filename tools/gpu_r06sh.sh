#!/bin/bash
# round 6: raw current-stream handle -- check, the GPU tests that use it, the training bench
set -o pipefail
mkdir -p gpurun_out/sh
timeout -k 10 120 python -u tools/stream_handle_check.py > gpurun_out/sh/check.txt 2>&1 && cat gpurun_out/sh/check.txt | tail -1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -o cache_dir=/tmp/pc > gpurun_out/sh/pytest.log 2>&1 && tail -1 gpurun_out/sh/pytest.log || exit 1
timeout -k 10 120 python -u tools/train_host_probe.py > gpurun_out/sh/host.txt 2>&1 && grep "per phase" gpurun_out/sh/host.txt
timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/sh/b.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/sh/b.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))"
