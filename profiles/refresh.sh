#!/bin/bash
# Round-end measurement refresh on one MI355X (from the repo root):  bash profiles/refresh.sh <tag>
# bench lines for every config (C3 also driver-style: --steps 20 --warmup 5) and the 8/4/2-rank shares (every rank's 8-rank
# C3 and C4 share too), BVH timings, kernel traces, rocprof stats + PMC passes.
# Every step has its own time limit; the first failure ends the script.
set -eo pipefail
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3_driver.json 2> $O/bench_c3_driver.err
for c in c2 c4 c5 c1; do timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err; done
for n in 8 4 2; do GSRT_DEBUG_RANK_OF=$n timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-stats > $O/bench_c3r$n.json 2> $O/bench_c3r$n.err; done
GSRT_DEBUG_RANK_OF=8 timeout -k 10 200 python3 bench.py --config c4 --no-cpu-baseline --no-stats > $O/bench_c4r8.json 2> $O/bench_c4r8.err
bash profiles/rank_shares_all.sh c3 8 $TAG > $O/rank_shares_c3r8.txt
bash profiles/rank_shares_all.sh c4 8 $TAG > $O/rank_shares_c4r8.txt
timeout -k 10 200 python3 profiles/bvh_timing.py > $O/bvh.txt 2>&1
bash profiles/traces.sh $TAG
bash profiles/collect.sh $TAG c3
echo refreshed
