# A/B of full builds with bench.py (sequential + pipelined, traced kernels): LIBS="a.so b.so"
set -e
for rep in 1 2; do for lib in $LIBS; do
  AA_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/bb.json 2>/dev/null
  python -c "
import json;d=json.load(open('gpurun_out/bb.json'))
print('rep$rep $(basename $lib)', 'pipe', round(d['value']), 'seq', round(d['sequential']['value']), {k:round(v['avg_ms']*1e3,2) for k,v in d['kernels'].items() if not k.startswith('k_gemm') and k != 'k_enc_heads3'})"
done; done
