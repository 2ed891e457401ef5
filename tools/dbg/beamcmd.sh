set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_beam.py > gpurun_out/beam_tests.log 2>&1
timeout -k 10 120 python bench_beam.py --no-cpu-baseline > gpurun_out/bb5.json
timeout -k 10 120 python bench_beam.py --no-cpu-baseline --tile128 > gpurun_out/bb4.json
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/beamprof -o beam -- python3 /root/repo/bench_beam.py --no-cpu-baseline --steps 5 > /root/repo/gpurun_out/beamprof.log 2>&1
