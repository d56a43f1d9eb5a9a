#!/bin/bash
# Multi-GPU estimate on one GPU: bench the share of rank 0 of an N-rank sharded C3 frame (GSRT_DEBUG_RANK_OF=N:
# its tiles, its tile groups, the full projection; no gather). value = the full frame's rays / that time,
# i.e. the N-GPU rate if every rank took as long as rank 0 and the gather were free.
set -e
CFG=${1:-c3}
mkdir -p gpurun_out
for n in 1 2 4 8; do
  GSRT_DEBUG_RANK_OF=$n timeout -k 10 120 python3 bench.py --config $CFG --no-cpu-baseline --no-stats > gpurun_out/rank_of_${CFG}_$n.log 2>&1
  echo "N=$n: $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"frame_ms_events": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/rank_of_${CFG}_$n.log | tr "\n" " ")"
done
