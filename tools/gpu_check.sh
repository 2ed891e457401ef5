#!/bin/bash
# One GPU call: the whole -m gpu suite, smoke, the default bench line and a rocprofv3 kernel summary
# of a short bench run.  Every GPU step has its own time limit; the script stops at the first crash
# or timeout.  usage: bash tools/gpu_check.sh <tag> [steps...]   steps: tests smoke bench prof (default all)
set -u
tag=${1:-run}; shift
steps=${@:-tests smoke bench prof}
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
for s in $steps; do
  case $s in
    tests) step tests timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest_gpu.log 2>&1
           grep -E "FAILED|ERROR|passed|failed" $out/pytest_gpu.log | tail -15 ;;
    smoke) step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
           tail -1 $out/smoke.log ;;
    bench) step bench timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
           python3 -c "import json;d=json.load(open('$out/bench.json'));e=d.get('eval_loop') or {};r=d['roofline'];print('value', round(d['value']), 'eval', round(e.get('value',0)), round(e.get('frac_of_value',0),3), 'pipe', round(d['pipelined']['value']), 'roofline', r['kernel'], round(r['frac'],3), round(r['avg_launch_ms']*1e3,2), 'us', {k: round(v['avg_ms']*1e3,2) for k,v in d['kernels'].items()})" ;;
    prof)  step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-eval-loop --pipeline-depth 1 --steps 20 > $out/prof.log 2>&1
           f=$(find $out/prof -name '*kernel_stats.csv' | head -1); head -14 "$f" | cut -c1-160 ;;
    train) step train timeout -k 10 300 python bench_train.py --no-cpu-baseline > $out/train_bench.json 2> $out/train_bench.err
           python3 -c "import json;a=json.load(open('$out/train_bench.json'));print('train', round(a['value'],1), 'steps/s')" ;;
    trainprof) step trainprof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_train -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 10 > $out/prof_train.log 2>&1
           f=$(find $out/prof_train -name '*kernel_stats.csv' | head -1); head -12 "$f" | cut -c1-140 ;;
    abenc) for r in 1 2; do for v in 1 0; do
             AA_ENC_V4=$v step abenc$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval-loop --pipeline-depth 1 --steps 20 > $out/ab_enc$v.$r.json 2>> $out/ab.err
             python3 -c "import json;d=json.load(open('$out/ab_enc$v.$r.json'));k=d['kernels'];print('AA_ENC_V4=$v', round(d['value']), 'enc', round(k['k_enc_v4']['avg_ms']*1e3,1), 'us')"
           done; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
