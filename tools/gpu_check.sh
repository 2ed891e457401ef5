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
           python3 -c "import json;a=json.load(open('$out/train_bench.json'));print('train', round(a['value'],1), 'steps/s', 'ms', round(a['ms_per_step'],3), 'host ms', round(a.get('host_ms_per_step',0),3))" ;;
    trainprof) step trainprof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_train -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 10 > $out/prof_train.log 2>&1
           f=$(find $out/prof_train -name '*kernel_stats.csv' | head -1); head -12 "$f" | cut -c1-140 ;;
    ab) # A/B of an environment switch: AB_VAR=name (values 0 / 1), two interleaved rounds of short bench runs
           for r in 1 2; do for v in 0 1; do
             env ${AB_VAR:-AA_ENC_REMAP}=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval-loop --steps 20 > $out/ab$v.$r.json 2>> $out/ab.err; rc=$?
             echo "[ab $v] exit $rc" >&3; [ $rc -eq 0 ] || exit $rc
             python3 -c "import json;d=json.load(open('$out/ab$v.$r.json'));k=d['kernels'];print('${AB_VAR:-AA_ENC_REMAP}=$v', round(d['value']), 'pipe', round(d['pipelined']['value']), {n: round(e['avg_ms']*1e3,2) for n,e in k.items()})"
           done; done ;;
    trainab) # A/B of an environment switch on the training bench: AB_VAR=name (0 / 1), two interleaved rounds
           for r in 1 2; do for v in 0 1; do
             env ${AB_VAR:-AA_TRA_ROW}=$v timeout -k 10 300 python bench_train.py --no-cpu-baseline > $out/trainab$v.$r.json 2>> $out/trainab.err; rc=$?
             echo "[trainab $v] exit $rc" >&3; [ $rc -eq 0 ] || exit $rc
             python3 -c "import json;a=json.load(open('$out/trainab$v.$r.json'));print('${AB_VAR:-AA_TRA_ROW}=$v train', round(a['value'],1), 'steps/s host ms', round(a.get('host_ms_per_step',0),3))"
           done; done ;;
    pipe) # pipelined-rate probe: depth 2/3/4 x slot streams raw/aux
           for ps in x; do for d in 2 3 4; do
             timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval-loop --no-trace --steps 20 --pipeline-depth $d > $out/pipe_${ps}_$d.json 2>> $out/pipe.err; rc=$?
             echo "[pipe $ps $d] exit $rc" >&3; [ $rc -eq 0 ] || exit $rc
             python3 -c "import json;d=json.load(open('$out/pipe_${ps}_$d.json'));print('streams $ps depth $d seq', round(d['value']), 'pipe', round(d['pipelined']['value']))"
           done; done ;;
    bits) # bitwise A/B of env switches on one training step (each switch: value 1 vs 0), bf16 and fp32
           for var in ${BITS_VARS:-AA_TRA_ROW AB_ONE_STREAM}; do for dt in bf16 fp32; do
             for v in 1 0; do
               env $var=$v timeout -k 10 300 python tools/ab_bits.py dump /tmp/bits_${var}_${dt}_$v.npz --train $dt --batch 128 --T 18 > $out/bits_${var}_$v.log 2>&1; rc=$?
               echo "[bits $var $dt $v] exit $rc" >&3; [ $rc -eq 0 ] || exit $rc
             done
             echo "== $var $dt"; python tools/ab_bits.py cmp /tmp/bits_${var}_${dt}_1.npz /tmp/bits_${var}_${dt}_0.npz > $out/bits_${var}_${dt}.cmp
             grep -E "DIFF|ALL BIT" $out/bits_${var}_${dt}.cmp | head -12; rm -f /tmp/bits_${var}_${dt}_*.npz
           done; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
