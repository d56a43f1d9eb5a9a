#!/bin/bash
# A/B timing of experiment builds (3dgs-raytrace_amd/gsrt/libgsrt_x*.so) against each other on one box:
#   bash profiles/ab.sh <config> <lib names...>     e.g. bash profiles/ab.sh c3 libgsrt_xbase libgsrt_x8
# Two interleaved rounds; one bench line per (lib, round) under gpurun_out/ab_<lib>_<round>.log.
set -e
CFG=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
  for lib in "$@"; do
    GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 120 python3 bench.py --config $CFG --no-cpu-baseline \
      > gpurun_out/ab_${lib}_$round.log 2>&1
    echo "$lib round $round: $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"frame_ms_events": [0-9.]*' gpurun_out/ab_${lib}_$round.log | tr "\n" " ")"
  done
done
