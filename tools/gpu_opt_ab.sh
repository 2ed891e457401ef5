set -o pipefail
mkdir -p gpurun_out/opt1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -o cache_dir=/tmp/pc > gpurun_out/opt1/pytest.log 2>&1; rc=$?; grep -E "FAIL|ERROR|passed|failed" gpurun_out/opt1/pytest.log | tail -25
[ $rc -le 1 ] || exit $rc
for v in "--opt torch --loss torch" "" "--opt torch --loss torch" ""; do
  timeout -k 10 200 python bench_train.py --no-cpu-baseline --steps 40 $v > gpurun_out/opt1/bt.json || exit $?
  python -c "import json;d=json.load(open('gpurun_out/opt1/bt.json'));print('$v', round(d['value'],1), round(d['ms_per_step'],3))"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/opt1/prof -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 10 > gpurun_out/opt1/prof.log 2>&1 || exit $?
exit $rc
