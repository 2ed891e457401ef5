#!/bin/bash
# round 6: persistent k_vexact (next tile's first K-step under the current tile's epilogue) --
# bitwise beams against the one-tile-per-workgroup build (abvar/vx0.so), the beam tests, A/B
set -o pipefail
mkdir -p gpurun_out/vx /tmp/abvx
AA_LIB_PATH=$PWD/abvar/vx0.so timeout -k 10 120 python -u tools/ab_bits.py dump /tmp/abvx/a.npz --beam 3 > /dev/null 2>> gpurun_out/vx/bits.err || exit 1
timeout -k 10 120 python -u tools/ab_bits.py dump /tmp/abvx/b.npz --beam 3 > /dev/null 2>> gpurun_out/vx/bits.err || exit 1
python3 tools/ab_bits.py cmp /tmp/abvx/a.npz /tmp/abvx/b.npz > gpurun_out/vx/bits.txt 2>&1; tail -1 gpurun_out/vx/bits.txt
rm -rf /tmp/abvx
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_beam.py > gpurun_out/vx/pytest.log 2>&1 && echo pytest-ok || exit 1
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export AA_LIB_PATH=$PWD/abvar/vx0.so; else unset AA_LIB_PATH; fi
    timeout -k 10 200 python -u bench_beam.py --no-cpu-baseline > gpurun_out/vx/b_${v}_${rep}.json 2>> gpurun_out/vx/b.err || exit 1
    echo "$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/vx/b_${v}_${rep}.json'));r=d.get('roofline',{});print(round(d['value']),round(d['ms_per_step'],3), r.get('median_launch_ms'), r.get('frac'))")"
  done
done
unset AA_LIB_PATH
