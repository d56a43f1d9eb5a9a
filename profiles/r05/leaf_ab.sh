#!/bin/bash
# A/B of the leaf-order projection threshold (GSRT_LEAF_ORDER_RANKS) on rank shares, then the exchange format on the
# 8-rank root share: bash profiles/r05/leaf_ab.sh <config> <libs...>   (lib "libgsrt" = the product build)
set -eo pipefail
CFG=$1; shift
O=gpurun_out/r05_leaf; mkdir -p $O
share() {  # lib N r extra-args...
  local lib=$1 N=$2 r=$3; shift 3
  local tag=$(echo "$*" | tr -c 'a-z0-9\n' '_')
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so GSRT_DEBUG_RANK_OF=$N:$r timeout -k 10 120 python3 bench.py --config $CFG \
    --no-cpu-baseline --no-stats --steps 300 --warmup 30 "$@" > $O/s_${lib}_${N}_$r$tag.json 2> $O/s_${lib}_${N}_$r.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ms', d['ms_per_step'], 'exch', d.get('rank_share_exchange_ms'))" \
    "$O/s_${lib}_${N}_$r$tag.json" "$lib N=$N r=$r $*"
}
for N in ${NS:-2 4 8}; do
  for lib in "$@"; do
    share $lib $N 0
    share $lib $N $((N - 1))
  done
done
share libgsrt 8 0 --out rgba32f
share libgsrt 8 0 --out dump8
