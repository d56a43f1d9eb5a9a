#!/bin/bash
# Every rank's share of an N-rank frame, each rendered alone on one GPU (GSRT_DEBUG_RANK_OF=N:r): the slowest share
# sets an N-GPU frame's period (before the gather). From the repo root on the GPU box:
#   bash profiles/rank_shares_all.sh <config> <N> [tag]
set -eo pipefail
CFG=$1; N=$2; TAG=${3:-rs}
O=gpurun_out/$TAG
mkdir -p $O
for ((r = 0; r < N; ++r)); do
  GSRT_DEBUG_RANK_OF=$N:$r timeout -k 10 120 python3 bench.py --config $CFG --no-cpu-baseline --no-stats \
    > $O/share_${CFG}_${N}_$r.json 2> $O/share_${CFG}_${N}_$r.err
  echo "$CFG N=$N rank $r: $(grep -o '"ms_per_step": [0-9.]*' $O/share_${CFG}_${N}_$r.json)"
done
