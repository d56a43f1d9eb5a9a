#!/bin/bash
# quick 1-GPU lines: bash profiles/r06/quick.sh <tag> <config>[:N:r] ...   (N:r = GSRT_DEBUG_RANK_OF rank share)
set -eo pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for spec in "$@"; do
  IFS=: read -r CFG N R <<< "$spec"
  if [ -n "$N" ]; then export GSRT_DEBUG_RANK_OF=$N:$R; else unset GSRT_DEBUG_RANK_OF; fi
  f=$O/${CFG}_${N:-1}_${R:-0}.json
  timeout -k 10 150 python3 bench.py --config $CFG --no-cpu-baseline --no-stats --steps 100 --warmup 20 $BENCH_EXTRA > $f 2> ${f%.json}.err
  python3 -c "import json; d=json.load(open('$f')); print('$spec', d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame')"
done
