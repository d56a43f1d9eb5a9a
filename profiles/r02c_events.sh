#!/bin/bash
# cost of the bench's per-frame HIP timing events (4 per frame on the render stream): with / without, two rounds
set -o pipefail
O=gpurun_out/events
mkdir -p $O
for spec in c3: c2: c4: c3:8; do
  cfg=${spec%%:*}; rk=${spec##*:}
  for r in 1 2; do for ev in "" "--no-events"; do
    if [ -n "$rk" ]; then export GSRT_DEBUG_RANK_OF=$rk; else unset GSRT_DEBUG_RANK_OF; fi
    timeout -k 10 150 python bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 5 $ev > $O/${cfg}_${rk}_${r}_${ev}.log 2>&1 || exit 1
    echo "$cfg/${rk:-1} [$ev] r$r: $(grep -o '"ms_per_step": [0-9.]*' $O/${cfg}_${rk}_${r}_${ev}.log)" >> $O/ab.log
  done; done
done
echo ok
