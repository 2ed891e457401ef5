set -e
cd /root/repo
for cfg in "256 128" "128 128" "128 256" "512 64" "0 128"; do
  set -- $cfg
  AA_TG_TARGET=$1 AA_TG_KMIN=$2 timeout -k 10 120 python bench_train.py --no-cpu-baseline --steps 30 > gpurun_out/tg_$1_$2.json
  echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/tg_$1_$2.json'));print(round(d['ms_per_step'],3))")"
done
