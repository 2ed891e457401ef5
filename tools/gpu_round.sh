#!/bin/bash
# One GPU call: the whole -m gpu suite, smoke, the training bench (HIP loss/Adam and torch's, A/B),
# a rocprofv3 kernel summary of the training bench and the default decode bench line.  Every GPU
# step has its own time limit; the script stops at the first crash or timeout.
# usage: bash tools/gpu_round.sh <tag>
set -u
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
exec 3>&1  # step reports go to the script's stdout even when a step's output is redirected
step() {  # name, then the command; stop unless it passed (0) or only had test failures (1)
  local name=$1; shift
  "$@"; local rc=$?
  echo "[$name] exit $rc" >&3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] crashed or timed out: stopping" >&3; exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest_gpu.log 2>&1
grep -E "FAILED|ERROR|passed|failed" $out/pytest_gpu.log | tail -12
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
step train timeout -k 10 300 python bench_train.py > $out/train_bench.json 2> $out/train_bench.err
step train_torch timeout -k 10 300 python bench_train.py --no-cpu-baseline --opt torch --loss torch > $out/train_bench_torch.json 2>> $out/train_bench.err
python3 -c "import json;a=json.load(open('$out/train_bench.json'));b=json.load(open('$out/train_bench_torch.json'));print('train hip', round(a['value'],1), 'torch', round(b['value'],1))"
step trainprof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_train -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 10 > $out/prof_train.log 2>&1
step bench timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
python3 -c "import json;d=json.load(open('$out/bench.json'));print('value', round(d['value']), 'pipe', round(d['pipelined']['value']), 'roofline', d['roofline']['kernel'], round(d['roofline']['frac'],3))"
