#!/bin/bash
# kernel durations of rank shares: overlapped (kernel trace) and alone (a PMC pass serialises the kernels)
#   bash profiles/r05/share_prof.sh <config> <N> <ranks...>  -> gpurun_out/r05/sp_<cfg>_<N>_<r>_{trace,alone}/
set -eo pipefail
CFG=$1; N=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
for r in "$@"; do
  B="bench.py --config $CFG --no-cpu-baseline --no-stats"
  GSRT_DEBUG_RANK_OF=$N:$r timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/sp_${CFG}_${N}_${r}_trace -o run -- python3 $B --steps 100 --warmup 20 > gpurun_out/r05/sp_${CFG}_${N}_${r}_trace.log 2>&1
  GSRT_DEBUG_RANK_OF=$N:$r timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/r05/sp_${CFG}_${N}_${r}_alone -o run -- python3 $B --steps 20 --warmup 5 --warmup-min-s 0 > gpurun_out/r05/sp_${CFG}_${N}_${r}_alone.log 2>&1
done
