set -u
mkdir -p gpurun_out/ce2
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_train.py tests/test_gpu_configs.py -v --timeout 200 --timeout-method thread -o cache_dir=/tmp/pc > gpurun_out/ce2/pytest.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/ce2/pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ce2/prof -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 10 > gpurun_out/ce2/prof.log 2>&1 || exit $?
timeout -k 10 300 python bench_train.py --no-cpu-baseline > gpurun_out/ce2/bt.json || exit $?
cat gpurun_out/ce2/bt.json | cut -c1-200
exit $rc
