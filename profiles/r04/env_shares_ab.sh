#!/bin/bash
# A/B of rank shares under different environment settings, two interleaved rounds (loopback exchange path):
#   bash profiles/r04/env_shares_ab.sh <config> <N> <rank> "<ENV=VAL ...>" ...   (N = 1: the whole frame on one GPU)
set -eo pipefail
CFG=$1; N=$2; R=$3; shift 3
O=gpurun_out/env_shares_ab
mkdir -p $O
for round in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i + 1))
    f=$O/${CFG}_${N}_${R}_${i}_$round
    if [ "$N" -gt 1 ]; then rk="GSRT_DEBUG_RANK_OF=$N:$R"; else rk="GSRT_UNUSED=0"; fi
    env $envs $rk timeout -k 10 120 python3 bench.py --config $CFG --no-cpu-baseline --no-stats --steps 200 --warmup 20 \
      > $f.json 2> $f.err
    python3 -c "import json; d=json.load(open('$f.json')); print('[$envs] $CFG N=$N rank $R round $round:', d['ms_per_step'], 'ms')"
  done
done
