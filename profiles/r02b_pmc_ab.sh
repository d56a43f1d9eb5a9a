#!/bin/bash
# PMC A/B of library builds on C3 (one counter pass per group, kernel trace only):
#   bash profiles/r02b_pmc_ab.sh <tag> <lib names...>
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
for lib in "$@"; do
  export GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so
  O=gpurun_out/pmc_$TAG/$lib
  mkdir -p $O
  B="bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 --warmup-min-s 0 --no-stats"
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O/sq2 -o run -- python3 $B > $O/sq2.log 2>&1 || exit 2
  timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $O/sq3 -o run -- python3 $B > $O/sq3.log 2>&1 || exit 3
done
echo ok
