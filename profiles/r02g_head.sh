#!/bin/bash
# Round-2 final HEAD refresh on one MI355X: driver-style bench of every config (+ the 8-rank shares and the 2- and
# 4-rank C3 shares), then the rocprof
# kernel-trace + PMC profile of C3 (profiles/collect.sh) summarised by parse_pmc.py
set -o pipefail
O=gpurun_out/${1:-r02d}
mkdir -p $O
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || exit 2
for c in c2 c4 c5 c1; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit 3
done
timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c3_100.log 2>&1 || exit 4
for c in c3 c4; do
  GSRT_DEBUG_RANK_OF=8 timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_${c}_rank8.log 2>&1 || exit 5
done
for r in 2 4; do
  GSRT_DEBUG_RANK_OF=$r timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_c3_rank$r.log 2>&1 || exit 5
done
bash profiles/collect.sh ${1:-r02d} c3 || exit 6
echo ok
