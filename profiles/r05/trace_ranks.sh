#!/bin/bash
# kernel traces of several rank shares (product build): bash profiles/r05/trace_ranks.sh <config> <N> <ranks...>
set -eo pipefail
CFG=$1; N=$2; shift 2
export TMPDIR=/tmp
O=gpurun_out/r05_trr; mkdir -p $O
for r in "$@"; do
  GSRT_DEBUG_RANK_OF=$N:$r timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${CFG}_${N}_$r -o run \
    -- python3 bench.py --config $CFG --no-cpu-baseline --no-stats --steps 200 --warmup 20 > $O/${CFG}_${N}_$r.json 2> $O/${CFG}_${N}_$r.err
  echo "rank $r: $(grep -o '"ms_per_step": [0-9.]*' $O/${CFG}_${N}_$r.json)"
done
