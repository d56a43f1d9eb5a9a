#!/bin/bash
# PMC passes of the C3 bench for experiment builds (3dgs-raytrace_amd/gsrt/libgsrt_x*.so), one rocprofv3 run per
# counter set (each within one block's limits) and library:
#   bash profiles/pmc_ab.sh <tag> <lib names...>      e.g. bash profiles/pmc_ab.sh smem libgsrt_xbase libgsrt_xsmem
# PMC_SETS picks the passes (default "sq sq2"; "fetch write" = the HBM byte counters). CFG picks the config (c3).
# Output under gpurun_out/pmc_<tag>/<lib>/{sq,sq2,sq3}; summarise with python profiles/pmc_summary.py <tag>.
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
SETS=${PMC_SETS:-sq sq2}
B="bench.py --config ${CFG:-c3} --no-cpu-baseline --steps 3 --warmup 1 --warmup-min-s 0 --no-stats"
for lib in "$@"; do
  OUT=gpurun_out/pmc_$TAG/$lib
  mkdir -p "$OUT"
  export GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so
  for set in $SETS; do
  case $set in
  fetch) timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- python3 $B > "$OUT/fetch.log" 2>&1 ;;
  write) timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- python3 $B > "$OUT/write.log" 2>&1 ;;
  sq) timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace --output-format csv -d "$OUT/sq" -o run -- python3 $B > "$OUT/sq.log" 2>&1 ;;
  sq2) timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq2" -o run -- python3 $B > "$OUT/sq2.log" 2>&1 ;;
  esac
  done
done
echo done
