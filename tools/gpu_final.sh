#!/bin/bash
# End-of-round evidence in one GPU call: the whole -m gpu suite, smoke, PMC traffic passes
# (FETCH_SIZE / WRITE_SIZE, separate runs) -> traffic.json, the default decode bench line (reads that
# traffic.json), a rocprofv3 kernel summary of the decode bench, the training bench + its rocprofv3
# summary, and the beam bench.  Every GPU step has its own time limit; the script stops at the first
# crash or timeout.  usage: bash tools/gpu_final.sh <tag>
set -u
tag=${1:-final}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
exec 3>&1
step() {  # name, then the command; stop unless it passed (0) or only had test failures (1)
  local name=$1; shift
  "$@"; local rc=$?
  echo "[$name] exit $rc" >&3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] crashed or timed out: stopping" >&3; exit $rc; fi
}
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest_gpu.log 2>&1
grep -E "FAILED|ERROR|passed|failed" $out/pytest_gpu.log | tail -8
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
for p in fetch write mfma; do
  step pmc_$p bash tools/pmc.sh $tag $p
done
python3 tools/pmc_summary.py gpurun_out/pmc_$tag --traffic $out/traffic.json > $out/pmc_traffic.txt 2>&1
python3 tools/mfma_util.py gpurun_out/pmc_$tag/mfma --json $out/mfma_util.json > $out/mfma_util.txt 2>&1
step bench timeout -k 10 600 python bench.py --traffic-json $out/traffic.json > $out/bench.json 2> $out/bench.err
python3 -c "import json;d=json.load(open('$out/bench.json'));print('value', round(d['value']), 'pipe', round(d['pipelined']['value']), 'eval', round(d['eval_loop']['value']), 'roofline', d['roofline']['kernel'], round(d['roofline']['frac'],3))"
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-trace --steps 10 > $out/prof.log 2>&1
step train timeout -k 10 300 python bench_train.py > $out/train_bench.json 2> $out/train_bench.err
python3 -c "import json;a=json.load(open('$out/train_bench.json'));print('train', round(a['value'],1))"
step trainprof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_train -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 10 > $out/prof_train.log 2>&1
step beam timeout -k 10 600 python bench_beam.py > $out/beam_bench.json 2> $out/beam_bench.err
python3 -c "import json;a=json.load(open('$out/beam_bench.json'));print('beam', round(a['value']))"
