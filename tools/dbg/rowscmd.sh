set -e
# r01_v13: beam-search (config 4) and training-step (config 5) benches of the current tree.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench_beam.py > gpurun_out/bench_beam.json 2> gpurun_out/bench_beam.err
head -c 300 gpurun_out/bench_beam.json; echo
timeout -k 10 300 python bench_train.py > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err
head -c 300 gpurun_out/bench_train.json; echo
