#!/bin/bash
# round 6: k_bgemm loading two K steps ahead (AA_BG_PF2, variant since removed) -- bitwise against the default, then interleaved A/B
set -o pipefail
mkdir -p gpurun_out/bgpf /tmp/abbg
for v in 0 1; do
  AA_BG_PF2=$v timeout -k 10 120 python -u tools/ab_bits.py dump /tmp/abbg/pf$v.npz --train bf16 > /dev/null 2>> gpurun_out/bgpf/bits.err || exit 1
done
python3 tools/ab_bits.py cmp /tmp/abbg/pf0.npz /tmp/abbg/pf1.npz > gpurun_out/bgpf/bits.txt 2>&1; tail -1 gpurun_out/bgpf/bits.txt
rm -rf /tmp/abbg
for rep in 1 2 3; do
  for v in 1 0; do
    AA_BG_PF2=$v timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/bgpf/b_${v}_${rep}.json 2>> gpurun_out/bgpf/b.err || exit 1
    echo "pf2=$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/bgpf/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
