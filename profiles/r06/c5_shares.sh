#!/bin/bash
# C5 rank shares through the loopback exchange path (update + refit + projection + lists + render + dump8 gather per
# frame), bands pinned from the whole frame's row profile as bench.py does, then one kernel trace of a share:
#   bash profiles/r06/c5_shares.sh <tag> <N> <trace rank|-> <ranks...>
set -eo pipefail
TAG=$1; N=$2; TR=$3; shift 3
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for r in "$@"; do
  GSRT_DEBUG_RANK_OF=$N:$r timeout -k 10 150 python3 bench.py --config c5 --no-cpu-baseline --no-stats --steps 100 --warmup 20 \
    > $O/share_c5_${N}_$r.json 2> $O/share_c5_${N}_$r.err
  python3 -c "import json; d=json.load(open('$O/share_c5_${N}_$r.json')); print('c5 N=$N rank $r:', d['ms_per_step'], 'ms, kernel', d.get('roofline',{}).get('kernel_ms'), 'exchange', d.get('rank_share_exchange_ms'), 'ms, bands', d.get('rank_share_bands'))"
done
if [ "$TR" != "-" ]; then
  GSRT_DEBUG_RANK_OF=$N:$TR timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5_${N}_$TR -o run \
    -- python3 bench.py --config c5 --no-cpu-baseline --no-stats --steps 100 --warmup 20 > $O/trace_c5_${N}_$TR.json 2> $O/trace_c5_${N}_$TR.err
  echo "trace rank $TR: $(grep -o '"ms_per_step": [0-9.]*' $O/trace_c5_${N}_$TR.json)"
fi
