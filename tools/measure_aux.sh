#!/bin/bash
# Config-4 (beam) and config-5 (training) measurement on one GPU box: bench line + rocprofv3 kernel
# stats for each.  Every GPU step has its own time limit; the script stops at the first failure.
# usage: bash tools/measure_aux.sh <tag>
set -u
tag=${1:-run}
out=gpurun_out/a_$tag
mkdir -p $out
export TMPDIR=/tmp
exec 3>&1  # step reports go to the script's stdout even when a step's output is redirected
run() { local name=$1; shift; "$@"; local rc=$?; echo "[$name] exit $rc" >&3; [ $rc -eq 0 ] || exit $rc; }
run beam timeout -k 10 300 python bench_beam.py > $out/beam.json 2> $out/beam.err
run beam_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/beam_prof -o run --output-format csv -- python3 bench_beam.py --no-cpu-baseline --steps 5 > $out/beam_prof.log 2>&1
run train timeout -k 10 300 python bench_train.py > $out/train.json 2> $out/train.err
run train_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/train_prof -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 10 > $out/train_prof.log 2>&1
python3 -c "
import json
for n in ('beam','train'):
    d=json.load(open('$out/'+n+'.json')); print(n, d['value'], d['unit'], json.dumps(d.get('roofline'))[:300])"
