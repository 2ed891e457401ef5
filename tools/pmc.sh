#!/bin/bash
# PMC passes over a short bench run (each pass its own rocprofv3 process; --kernel-trace/--stats only).
# usage: [PMC_CMD='python3 prog.py args'] bash tools/pmc.sh <tag> [pass...]   passes: sq mfma fetch write lds l2
set -u
tag=${1:-run}; shift
passes=${@:-sq fetch write}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$tag
for p in $passes; do
  case $p in
    sq)    ctr="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" ;;
    mfma)  ctr="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" ;;
    fetch) ctr="FETCH_SIZE" ;;
    write) ctr="WRITE_SIZE" ;;
    lds)   ctr="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL" ;;
    l2)    ctr="TCC_HIT_sum TCC_MISS_sum" ;;
    *) echo "unknown pass $p"; exit 2 ;;
  esac
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc_$tag/$p -o run -- \
     ${PMC_CMD:-python3 bench.py --no-cpu-baseline --no-trace --steps 2 --warmup 1} > gpurun_out/pmc_$tag/$p.log 2>&1
  rc=$?; echo "[pmc $p] exit $rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmc_$tag/$p.log; exit $rc; fi
done
