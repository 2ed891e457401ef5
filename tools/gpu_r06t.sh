#!/bin/bash
# round 6: Adam plan reuse + HIP clip_grad_norm_ (tests, training bench, host probes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_train.py tests/test_gpu_configs.py > gpurun_out/t_pytest.log 2>&1 && echo pytest-ok &&
timeout -k 10 120 python -u bench_train.py --no-cpu-baseline > gpurun_out/t_bench.json 2> gpurun_out/t_bench.err && echo bench-ok &&
timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --opt torch > gpurun_out/t_bench_torchopt.json 2>> gpurun_out/t_bench.err && echo bench2-ok &&
timeout -k 10 120 python -u tools/train_host_probe.py > gpurun_out/t_host.txt 2>&1 && echo host-ok &&
timeout -k 10 120 python -u tools/train_ccall_probe.py > gpurun_out/t_ccall.txt 2>&1 && echo ccall-ok
