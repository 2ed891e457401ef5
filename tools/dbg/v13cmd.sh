set -e
# r01_v13: GPU tests, smoke, default bench, rocprofv3 stats and PMC traffic of the current tree.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
head -c 400 gpurun_out/bench.json; echo
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/benchprof -o bench -- python3 /root/repo/bench.py --no-cpu-baseline --steps 10 > /root/repo/gpurun_out/benchprof.log 2>&1
cd /root/repo
bash tools/pmc.sh traffic fetch write
python tools/pmc_summary.py gpurun_out/pmc_traffic --traffic gpurun_out/traffic.json > gpurun_out/pmc_traffic/summary.txt 2>&1
head -30 gpurun_out/pmc_traffic/summary.txt
