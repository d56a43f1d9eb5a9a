#!/bin/bash
# gather / unpack stream split A/B, two interleaved rounds: GSRT_COMM_SPLIT=0, =1, =1 with GPU_MAX_HW_QUEUES=8
set -eo pipefail
for round in 1 2; do
  for v in 0 1 1q; do
    if [ $v = 1q ]; then export GPU_MAX_HW_QUEUES=8 GSRT_COMM_SPLIT=1; else unset GPU_MAX_HW_QUEUES; export GSRT_COMM_SPLIT=$v; fi
    echo "== round $round split $v"
    bash profiles/r04/shares.sh split${v}_$round c3 8 0 4
    bash profiles/r04/shares.sh split${v}_$round c4 8 0 4
  done
done
