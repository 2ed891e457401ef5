#!/bin/bash
# Round measurement on one GPU box: GPU tests, smoke, the default bench line, rocprofv3 kernel stats,
# PMC traffic (FETCH/WRITE) and MFMA-busy passes.  Every GPU step has its own time limit and the
# script stops at the first crash or timeout.  usage: bash tools/measure.sh <tag>
set -u
tag=${1:-run}
out=gpurun_out/m_$tag
mkdir -p $out
export TMPDIR=/tmp
exec 3>&1  # step reports go to the script's stdout even when a step's output is redirected
step() {  # name, then the command; stop unless it passed (0) or only had test failures (1)
  local name=$1; shift
  "$@"; local rc=$?
  echo "[$name] exit $rc" >&3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] crashed or timed out: stopping" >&3; exit $rc; fi
}
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest_gpu.log 2>&1
tail -3 $out/pytest_gpu.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
step bench timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-trace --steps 10 > $out/prof.log 2>&1
for p in fetch write mfma; do
  step pmc_$p bash tools/pmc.sh m_$tag $p
done
python3 tools/pmc_summary.py gpurun_out/pmc_m_$tag --traffic $out/traffic.json > $out/pmc_traffic.txt 2>&1
python3 tools/mfma_util.py gpurun_out/pmc_m_$tag/mfma --json $out/mfma_util.json > $out/mfma_util.txt 2>&1
python3 -c "import json;d=json.load(open('$out/bench.json'));print('value', round(d['value']), 'pipe', round(d['pipelined']['value']), 'roofline', d['roofline']['kernel'], round(d['roofline']['frac'],3))"
