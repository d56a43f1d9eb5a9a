#!/bin/bash
# binned group lists A/B (GSRT_BINS=1 default vs 0 = per-group BVH traversal), two interleaved rounds:
# 8-rank C3 / C4 shares of ranks 0 and 4, and whole C3 / C2 frames. bash profiles/r04/bins_ab.sh <tag>
set -eo pipefail
TAG=${1:-bins}
O=gpurun_out/$TAG
mkdir -p $O
for round in 1 2; do
  for v in 1 0; do
    export GSRT_BINS=$v
    echo "== round $round GSRT_BINS=$v"
    bash profiles/r04/shares.sh ${TAG}_${v}_$round c3 8 0 4
    bash profiles/r04/shares.sh ${TAG}_${v}_$round c4 8 0 4
    for c in c3 c2; do
      timeout -k 10 120 python3 bench.py --config $c --steps 100 --warmup 20 --no-cpu-baseline --no-stats > $O/${c}_${v}_$round.json 2> $O/${c}_${v}_$round.err
      python3 -c "import json; d=json.load(open('$O/${c}_${v}_$round.json')); print('$c', d['value'], 'Mrays/s', d['ms_per_step'], 'ms')"
    done
  done
done
