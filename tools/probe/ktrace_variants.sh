# ktrace over several instrumented builds: LIBS="tools/_build/lib_ts.so ..." [KT_ARGS=...]
set -e
for lib in $LIBS; do
  echo "== $(basename $lib)"
  AA_LIB_PATH=$PWD/$lib timeout -k 5 120 python tools/ktrace.py $KT_ARGS > gpurun_out/kt.log 2>&1 || { tail -5 gpurun_out/kt.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/kt.log
done
