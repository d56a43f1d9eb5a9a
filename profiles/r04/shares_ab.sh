#!/bin/bash
# A/B of rank shares through the loopback sharded path, two interleaved rounds:
#   bash profiles/r04/shares_ab.sh <config> <N> <rank> <lib names...>   (libraries in 3dgs-raytrace_amd/gsrt/)
set -eo pipefail
CFG=$1; N=$2; R=$3; shift 3
O=gpurun_out/shares_ab
mkdir -p $O
for round in 1 2; do
  for lib in "$@"; do
    f=$O/${lib}_${CFG}_${N}_${R}_$round
    GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so GSRT_DEBUG_RANK_OF=$N:$R timeout -k 10 120 python3 bench.py --config $CFG \
      --no-cpu-baseline --no-stats --steps 200 --warmup 20 > $f.json 2> $f.err
    python3 -c "import json; d=json.load(open('$f.json')); print('$lib $CFG N=$N rank $R round $round:', d['ms_per_step'], 'ms')"
  done
done
