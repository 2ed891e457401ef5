#!/bin/bash
# Round 6, first GPU call: the whole -m gpu suite on the working tree (ADVICE r5 fixes), the
# write-through-store A/B (abvar/wt0..wt4.so, tools/ab.sh, sequential decode), the beam A/B of this
# tree against the round-4 tree (abvar/r04m_tree, built in place) on ONE box, and the N = 2 gloo
# rehearsal of bench.py's multi-rank line (rank topology + neighbour-shard cross-check).
# Every GPU step has its own time limit; the script stops at the first crash or timeout.
set -u
out=gpurun_out/r06a
mkdir -p $out
step() {  # name, then the command; stop unless it passed (0) or only had test failures (1)
  local name=$1; shift
  "$@"; local rc=$?
  echo "[$name] exit $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] crashed or timed out: stopping"; exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -o cache_dir=/tmp/pc > $out/pytest_gpu.log 2>&1
tail -3 $out/pytest_gpu.log
LIBS="abvar/wt0.so abvar/wt1.so abvar/wt2.so abvar/wt3.so abvar/wt4.so" step ab timeout -k 10 900 bash tools/ab.sh --no-eval-loop --pipeline-depth 1 --steps 20 > $out/ab_wt.txt 2>&1
cat $out/ab_wt.txt
for rep in 1 2; do
  step beam_head$rep timeout -k 10 300 python bench_beam.py --no-cpu-baseline > $out/beam_head$rep.json 2> $out/beam_head$rep.err
  step beam_r04m$rep bash -c "cd abvar/r04m_tree && timeout -k 10 300 python bench_beam.py --no-cpu-baseline > ../../$out/beam_r04m$rep.json 2> ../../$out/beam_r04m$rep.err"
  python3 - $out/beam_head$rep.json $out/beam_r04m$rep.json <<'EOF'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f, round(d["value"]), "k_vexact_ms", round(d["roofline"]["avg_launch_ms"], 4), "frac", round(d["roofline"]["frac"], 3))
EOF
done
AA_DIST_BACKEND=gloo step n2 timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline --no-trace --no-eval-loop --pipeline-depth 1 --steps 5 > $out/bench_n2_gloo.json 2> $out/bench_n2_gloo.err
python3 -c "import json;d=json.load(open('$out/bench_n2_gloo.json'));print('n2', d['ranks_seen'], d['backend'], d['rank_devices'], d['cross_check'])"
