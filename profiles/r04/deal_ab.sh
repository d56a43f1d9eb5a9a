#!/bin/bash
# Deal variants over every rank of an N-rank share (loopback exchange path), variants interleaved per rank:
#   bash profiles/r04/deal_ab.sh <config> <N> "<lib>[:<root share>]" ...   (root share: GSRT_ROOT_SHARE, optional)
set -eo pipefail
CFG=$1; N=$2; shift 2
O=gpurun_out/deal_ab
mkdir -p $O
for ((r = 0; r < N; r++)); do
  for spec in "$@"; do
    lib=${spec%%:*}; w=""; [[ $spec == *:* ]] && w=${spec##*:}
    f=$O/${lib}_w${w:-def}_${CFG}_${N}_$r
    env ${w:+GSRT_ROOT_SHARE=$w} GSRT_DEBUG_RANK_OF=$N:$r GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 120 \
      python3 bench.py --config $CFG --no-cpu-baseline --no-stats --steps 200 --warmup 20 > $f.json 2> $f.err
    python3 -c "import json; d=json.load(open('$f.json')); print('$spec $CFG N=$N rank $r:', d['ms_per_step'], 'ms')"
  done
done
