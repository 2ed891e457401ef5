#!/bin/bash
# Round-5 measurement call: decode GPU tests (parity, pipeline), the default bench line, then a
# rocprofv3 kernel trace of the SAME sequential region the bench's roofline is timed on (bench.py
# --no-trace --pipeline-depth 1 --no-eval-loop: sampler() calls one after another, nothing else),
# summarised per kernel with medians by tools/kstats.py.  Every GPU step has its own time limit; the
# script stops at the first crash or timeout.  usage: bash tools/gpu_r05.sh <tag> [tests]
set -u
tag=${1:-r05}
tests=${2:-tests/test_gpu_parity.py tests/test_gpu_pipeline.py}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
exec 3>&1
step() {
  local name=$1; shift
  "$@"; local rc=$?
  echo "[$name] exit $rc" >&3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] crashed or timed out: stopping" >&3; exit $rc; fi
}
if [ "$tests" != none ]; then
  step tests timeout -k 10 600 python -u -m pytest $tests -m gpu -x -q --timeout 200 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest.log 2>&1
  tail -3 $out/pytest.log
fi
step bench timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err
python3 - "$out/bench.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 4), "traced", round(d["traced_ms_per_step"], 4),
      "ksum", round(d["kernel_sum_ms_per_step"], 4), "pipe", round(d["pipelined"]["value"]))
print("roofline", r["kernel"], "frac", round(r["frac"], 4), "median_us", round(r["median_launch_ms"] * 1e3, 2))
for k, v in d["kernels"].items():
    print(f"  {k:16s} med {v['median_ms']*1e3:7.2f}  mean {v['avg_ms']*1e3:7.2f}  n {v['launches']}")
EOF
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-trace --no-eval-loop --pipeline-depth 1 --steps 20 > $out/prof.log 2>&1
kt=$(find $out/prof -name "*kernel_trace.csv" | head -1)
[ -n "$kt" ] && python3 tools/kstats.py "$kt" $out/kernel_durations.csv
exit 0
