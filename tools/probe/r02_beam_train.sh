# round-2 measurements of the beam (config 4) and training (config 5) benches + rocprof/PMC summaries
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r02bt
timeout -k 10 300 python bench_beam.py > gpurun_out/r02bt/beam.json 2> gpurun_out/r02bt/beam.err
timeout -k 10 300 python bench_beam.py --fast --no-cpu-baseline > gpurun_out/r02bt/beam_fast.json 2> gpurun_out/r02bt/beam_fast.err
timeout -k 10 300 python bench_train.py > gpurun_out/r02bt/train.json 2> gpurun_out/r02bt/train.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02bt/prof_beam -o run --output-format csv -- python3 bench_beam.py --no-cpu-baseline --steps 3 > gpurun_out/r02bt/prof_beam.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02bt/prof_train -o run --output-format csv -- python3 bench_train.py --no-cpu-baseline --steps 5 > gpurun_out/r02bt/prof_train.log 2>&1
PMC_CMD="python3 bench_beam.py --no-cpu-baseline --steps 2 --warmup 1" bash tools/pmc.sh beam fetch write
python tools/pmc_summary.py gpurun_out/pmc_beam --traffic gpurun_out/r02bt/traffic_beam.json > gpurun_out/r02bt/pmc_beam.txt
echo done
