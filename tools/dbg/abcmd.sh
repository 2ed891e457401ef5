set -e
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/ab_tests.log 2>&1 || echo "tests failed (see log)"
for rep in 1 2; do
for lib in new old; do
  if [ $lib = old ]; then export AA_LIB_PATH=/root/repo/tools/_build/lib_old.so; else unset AA_LIB_PATH; fi
  for d in 2 4; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-trace --steps 100 --pipeline-depth $d > gpurun_out/ab.json
    echo "rep$rep $lib depth $d $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(round(d['value']), round(d['ms_per_step'],4), round(d['sequential']['value']))")"
  done
done
done
