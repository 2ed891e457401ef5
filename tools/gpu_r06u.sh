#!/bin/bash
# round 6: k_tgemm128 (128 x 128 training GEMM tiles) -- parity, then an interleaved A/B against the
# 64 x 64 engine (AA_TG128=0), then a kernel trace of the new default
set -o pipefail
mkdir -p gpurun_out/u
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_configs.py tests/test_gpu_optim.py > gpurun_out/u/pytest.log 2>&1 && echo pytest-ok || exit 1
for rep in 1 2 3; do
  for v in 1 0; do
    AA_TG128=$v timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 200 > gpurun_out/u/b_${v}_${rep}.json 2>> gpurun_out/u/b.err || exit 1
    echo "tg128=$v rep=$rep $(python3 -c "import json;d=json.load(open('gpurun_out/u/b_${v}_${rep}.json'));print(round(d['value'],1),round(d['ms_per_step'],3),round(d['host_ms_per_step'],3))")"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/u/prof -o run -- python3 $GRAFT_REPO_ROOT/bench_train.py --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/u/prof.log 2>&1 && echo prof-ok
