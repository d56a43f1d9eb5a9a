#!/bin/bash
# env-knob A/B on one box, two interleaved rounds:  bash profiles/r02b_env_ab.sh <config> "<envA>" "<envB>" ...
# (an env string may hold several VAR=value words; GSRT_DEBUG_RANK_OF=8 measures rank 0's share of 8)
set -o pipefail
CFG=$1; shift
mkdir -p gpurun_out/env_ab
for round in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline > gpurun_out/env_ab/${CFG}_${i}_$round.log 2>&1 || exit 1
    echo "$CFG [$e] r$round: $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frame_ms_events": [0-9.]*' gpurun_out/env_ab/${CFG}_${i}_$round.log | tr "\n" " ")"
  done
done
