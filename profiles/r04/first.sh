#!/bin/bash
# round-4 first GPU pass: the -m gpu suite, the C3 bench, and rank 0 / rank 4 shares of the 8-rank C3 and C4 frames
# through the loopback sharded path
set -eo pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3_driver.json 2> $O/bench_c3_driver.err
for spec in 8 8:4; do
  GSRT_DEBUG_RANK_OF=$spec timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-stats > $O/share_c3_${spec/:/_}.json 2> $O/share_c3_${spec/:/_}.err
  GSRT_DEBUG_RANK_OF=$spec timeout -k 10 120 python3 bench.py --config c4 --no-cpu-baseline --no-stats > $O/share_c4_${spec/:/_}.json 2> $O/share_c4_${spec/:/_}.err
done
echo done
