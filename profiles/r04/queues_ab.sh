#!/bin/bash
# Hardware queues per process (GPU_MAX_HW_QUEUES) against stream schemes, two interleaved rounds:
#   bash profiles/r04/queues_ab.sh <config> <N> <rank> "<lib>:<queues>" ...   (N = 1: the whole frame on one GPU)
set -eo pipefail
CFG=$1; N=$2; R=$3; shift 3
O=gpurun_out/queues_ab
mkdir -p $O
for round in 1 2; do
  for spec in "$@"; do
    lib=${spec%%:*}; q=${spec##*:}
    f=$O/${lib}_q${q}_${CFG}_${N}_${R}_$round
    if [ "$N" -gt 1 ]; then export GSRT_DEBUG_RANK_OF=$N:$R; else unset GSRT_DEBUG_RANK_OF; fi
    GPU_MAX_HW_QUEUES=$q GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 120 python3 bench.py --config $CFG \
      --no-cpu-baseline --no-stats --steps 200 --warmup 20 > $f.json 2> $f.err
    python3 -c "import json; d=json.load(open('$f.json')); print('$lib queues $q $CFG N=$N rank $R round $round:', d['ms_per_step'], 'ms')"
  done
done
