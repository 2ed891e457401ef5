set -e
cd /root/repo
for rep in 1 2; do
for cap in 0 128 64; do
  AA_ENC_WG=$cap timeout -k 10 120 python bench.py --no-cpu-baseline --no-trace --steps 100 --pipeline-depth 4 > gpurun_out/cap.json
  echo "rep$rep cap $cap $(python -c "import json;d=json.load(open('gpurun_out/cap.json'));print(round(d['value']), round(d['ms_per_step'],4), round(d['sequential']['value']))")"
done
done
AA_ENC_WG=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "encoder or golden" > gpurun_out/cap_tests.log 2>&1 || echo "cap tests failed"
