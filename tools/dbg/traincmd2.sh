set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py > gpurun_out/train_tests.log 2>&1
timeout -k 10 120 python bench_train.py --no-cpu-baseline --steps 30 > gpurun_out/bt_bf16.json
timeout -k 10 120 python bench_train.py --no-cpu-baseline --steps 30 --dtype fp32 > gpurun_out/bt_fp32.json
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/trainprof2 -o train -- python3 /root/repo/bench_train.py --no-cpu-baseline --steps 8 > /root/repo/gpurun_out/trainprof.log 2>&1
