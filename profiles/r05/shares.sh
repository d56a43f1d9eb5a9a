#!/bin/bash
# rank shares through the loopback sharded path (bands pinned from the whole frame's row profile, as bench.py does):
#   bash profiles/r05/shares.sh <tag> <config> <N> <ranks...>     (GSRT_LIB_PATH passes through)
set -eo pipefail
TAG=$1; CFG=$2; N=$3; shift 3
O=gpurun_out/$TAG
mkdir -p $O
for r in "$@"; do
  GSRT_DEBUG_RANK_OF=$N:$r timeout -k 10 120 python3 bench.py --config $CFG --no-cpu-baseline --no-stats --steps 200 --warmup 20 \
    > $O/share_${CFG}_${N}_$r.json 2> $O/share_${CFG}_${N}_$r.err
  python3 -c "import json; d=json.load(open('$O/share_${CFG}_${N}_$r.json')); print('$CFG N=$N rank $r:', d['ms_per_step'], 'ms, exchange', d.get('rank_share_exchange_ms'), 'ms, bands', d.get('rank_share_bands'))"
done
