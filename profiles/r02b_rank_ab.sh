#!/bin/bash
# rank-0 share of an 8-rank sharded frame (GSRT_DEBUG_RANK_OF=8) under env A/B knobs, two interleaved rounds:
#   bash profiles/r02b_rank_ab.sh <config> "<envA>" "<envB>" ...
set -o pipefail
CFG=$1; shift
mkdir -p gpurun_out/rank_ab
for round in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env GSRT_DEBUG_RANK_OF=8 $e timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline > gpurun_out/rank_ab/${CFG}_${i}_$round.log 2>&1 || exit 1
    echo "[$e] round $round: $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frame_ms_events": [0-9.]*' gpurun_out/rank_ab/${CFG}_${i}_$round.log | tr "\n" " ")"
  done
done
