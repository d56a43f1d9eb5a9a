#!/bin/bash
# rank_share.sh for several builds: bash profiles/rank_share_ab.sh <config> <N> <lib names...>
set -e
CFG=$1; N=$2; shift 2
mkdir -p gpurun_out
for round in 1 2; do
  for lib in "$@"; do
    GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so GSRT_DEBUG_RANK_OF=$N timeout -k 10 120 python3 bench.py --config $CFG \
      --no-cpu-baseline --no-stats > gpurun_out/rsab_${lib}_${N}_$round.log 2>&1
    echo "$lib N=$N round $round: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/rsab_${lib}_${N}_$round.log | tr "\n" " ")"
  done
done
