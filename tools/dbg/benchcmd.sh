set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/pipe_tests.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/benchprof -o bench -- python3 /root/repo/bench.py --no-cpu-baseline > /root/repo/gpurun_out/benchprof.log 2>&1
