#!/bin/bash
# GPU-box driver: every GPU step under its own timeout; stop at the first crash/timeout.
# usage: bash run_gpu.sh <step>...   steps: smoke tests testsall bench benchq prof pmc beamtests beambench beamprof
set -u
mkdir -p gpurun_out
ok_or_fail() {  # continue on 0 (pass) or 1 (test failures); stop on crashes/timeouts
  local rc=$1 name=$2
  echo "[$name] exit $rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[$name] crashed/timed out -> stopping"; exit "$rc"; fi
}
for step in "$@"; do
  case "$step" in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok_or_fail $? smoke; tail -3 gpurun_out/smoke.log ;;
    one) timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py} -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_one.log 2>&1; ok_or_fail $? one; tail -30 gpurun_out/pytest_one.log ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; ok_or_fail $? tests; tail -15 gpurun_out/pytest_gpu.log ;;
    testsall) timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; ok_or_fail $? tests; tail -25 gpurun_out/pytest_gpu.log ;;
    bench) timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; ok_or_fail $? bench; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err ;;
    benchq) timeout -k 10 600 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench.json 2> gpurun_out/bench.err; ok_or_fail $? bench; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err ;;
    lanes) for n in 1 2 3 4; do timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --lanes $n ${LANES_ARGS:-} > gpurun_out/bench_l$n.json 2>> gpurun_out/bench.err; ok_or_fail $? lanes$n; python -c "import json;d=json.load(open('gpurun_out/bench_l$n.json'));print('lanes $n', round(d['value']), 'captions/s', round(d['ms_per_step'],3),'ms')"; done ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-trace --steps 10 > gpurun_out/prof.log 2>&1; ok_or_fail $? prof ;;
    pmc)  bash tools/pmc.sh traffic fetch write; ok_or_fail $? pmc
          python tools/pmc_summary.py gpurun_out/pmc_traffic --traffic gpurun_out/traffic.json > gpurun_out/pmc_traffic/summary.txt 2>&1; cat gpurun_out/pmc_traffic/summary.txt ;;
    beamtests) timeout -k 10 600 python -m pytest tests/test_gpu_beam.py -m gpu -q > gpurun_out/pytest_beam.log 2>&1; ok_or_fail $? beamtests; tail -25 gpurun_out/pytest_beam.log ;;
    beambench) timeout -k 10 600 python bench_beam.py > gpurun_out/bench_beam.json 2> gpurun_out/bench_beam.err; ok_or_fail $? beambench; cat gpurun_out/bench_beam.json; tail -5 gpurun_out/bench_beam.err ;;
    beamprof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_beam -o run --output-format csv -- python bench_beam.py --no-cpu-baseline --steps 5 > gpurun_out/prof_beam.log 2>&1; ok_or_fail $? beamprof ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
