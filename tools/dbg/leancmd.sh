set -e
cd /root/repo
AA_LEAN_LSTM=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/lean_tests.log 2>&1 || echo "lean tests failed (see log)"
for rep in 1 2; do
for lean in 0 1; do
for d in 2 4; do
  AA_LEAN_LSTM=$lean timeout -k 10 120 python bench.py --no-cpu-baseline --no-trace --steps 100 --pipeline-depth $d > gpurun_out/lean.json
  echo "rep$rep lean=$lean depth $d $(python -c "import json;d=json.load(open('gpurun_out/lean.json'));print(round(d['value']), round(d['ms_per_step'],4), round(d['sequential']['value']))")"
done
done
done
cd /tmp && AA_LEAN_LSTM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/leanprof -o lean -- python3 /root/repo/bench.py --no-cpu-baseline --no-trace --steps 20 > /root/repo/gpurun_out/leanprof.log 2>&1
