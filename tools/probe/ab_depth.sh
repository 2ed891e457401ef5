# A/B of builds at several pipeline depths (distinct feature buffers): LIBS="a.so b.so" DEPTHS="2 4"
set -e
for rep in 1 2; do for lib in $LIBS; do for D in ${DEPTHS:-2 4}; do
  AA_LIB_PATH=$PWD/$lib timeout -k 10 150 python bench.py --no-cpu-baseline --no-trace --steps 40 --pipeline-depth $D > gpurun_out/bb.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/bb.json'));print('rep$rep $(basename $lib) depth', $D, 'pipe', round(d['value']), 'seq', round(d['sequential']['value']))"
done; done; done
