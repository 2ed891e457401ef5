#!/bin/bash
# round 6: training GEMM attribution -- shapes of one step (AA_TG_LOG) and a kernel trace of the
# 64 x 64 engine (AA_TG128=0) and of the 128 x 128 one
set -o pipefail
mkdir -p gpurun_out/v
AA_TG_LOG=1 timeout -k 10 120 python -u bench_train.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/v/log.json 2> gpurun_out/v/tglog.txt || exit 1
cd /tmp && export TMPDIR=/tmp
AA_TG128=0 timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/v/prof0 -o run -- python3 $GRAFT_REPO_ROOT/bench_train.py --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/v/prof0.log 2>&1 && echo prof0-ok || exit 1
AA_TG128=1 timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/v/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench_train.py --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/v/prof1.log 2>&1 && echo prof1-ok
