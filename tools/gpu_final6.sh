#!/bin/bash
# End-of-round evidence in one GPU call (round 6): the whole -m gpu suite, smoke, PMC traffic and
# MFMA-busy passes (separate rocprofv3 runs, --kernel-trace only beside --pmc) -> traffic.json, the
# default decode bench line (reading that traffic.json), a rocprofv3 kernel trace of the SAME
# sequential region the line's roofline is timed on, summarised per kernel with medians
# (tools/kstats.py), the training bench + its kernel trace, and the beam bench.  Every GPU step has
# its own time limit; the script stops at the first crash or timeout.  usage: bash tools/gpu_final6.sh <tag>
set -u
tag=${1:-r06z}
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
grep -E "FAILED|ERROR|passed|failed" $out/pytest_gpu.log | tail -4
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
export PMC_CMD="python3 bench.py --no-cpu-baseline --no-trace --no-eval-loop --pipeline-depth 1 --steps 2 --warmup 1"
for p in fetch write mfma; do
  step pmc_$p bash tools/pmc.sh $tag $p
done
python3 tools/pmc_summary.py gpurun_out/pmc_$tag --traffic $out/traffic.json > $out/pmc_traffic.txt 2>&1
python3 tools/mfma_util.py gpurun_out/pmc_$tag/mfma --json $out/mfma_util.json > $out/mfma_util.txt 2>&1
step bench timeout -k 10 600 python bench.py --traffic-json $out/traffic.json > $out/bench.json 2> $out/bench.err
python3 - $out/bench.json <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 4), "ksum", round(d["kernel_sum_ms_per_step"], 4),
      "pipe", round(d["pipelined"]["value"]), "eval", round(d["eval_loop"]["value"]), "cpu", round(d["cpu_baseline"]["value"]))
print("roofline", r["kernel"], "frac", round(r["frac"], 4), "median_us", round(r["median_launch_ms"] * 1e3, 2), "traffic", r["traffic"])
EOF
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-trace --no-eval-loop --pipeline-depth 1 --steps 20 > $out/prof.log 2>&1
kt=$(find $out/prof -name "*kernel_trace.csv" | head -1)
[ -n "$kt" ] && python3 tools/kstats.py "$kt" $out/kernel_durations.csv | head -12
step train timeout -k 10 300 python bench_train.py > $out/train_bench.json 2> $out/train_bench.err
python3 -c "import json;a=json.load(open('$out/train_bench.json'));print('train', round(a['value'],1))"
step trainprof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_train -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 10 > $out/prof_train.log 2>&1
kt=$(find $out/prof_train -name "*kernel_trace.csv" | head -1)
[ -n "$kt" ] && python3 tools/kstats.py "$kt" $out/train_kernel_durations.csv > /dev/null
step beam timeout -k 10 600 python bench_beam.py > $out/beam_bench.json 2> $out/beam_bench.err
python3 -c "import json;a=json.load(open('$out/beam_bench.json'));print('beam', round(a['value']))"
step n2 env AA_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline --no-trace --no-eval-loop --pipeline-depth 1 --steps 5 > $out/bench_n2_gloo.json 2> $out/bench_n2_gloo.err
python3 -c "import json;d=[json.loads(l) for l in open('$out/bench_n2_gloo.json') if l.startswith('{')][0];print('n2', d['ranks_seen'], d['backend'], d['cross_check']['ok'])"
