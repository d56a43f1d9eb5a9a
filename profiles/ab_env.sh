#!/bin/bash
# A/B timing of one library under different environment settings, two interleaved rounds:
#   bash profiles/ab_env.sh <config> "<ENV=VAL ...>" "<ENV=VAL ...>" ...     e.g. ... c3 "GSRT_PARTS=1" "GSRT_PARTS=4"
set -e
CFG=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i + 1))
    env $envs timeout -k 10 120 python3 bench.py --config $CFG --no-cpu-baseline > gpurun_out/abe_${CFG}_${i}_$round.log 2>&1
    echo "[$envs] round $round: $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"frame_ms_events": [0-9.]*' gpurun_out/abe_${CFG}_${i}_$round.log | tr "\n" " ")"
  done
done
