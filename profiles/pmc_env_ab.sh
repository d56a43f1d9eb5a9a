#!/bin/bash
# HBM byte counters (FETCH_SIZE, WRITE_SIZE: one rocprofv3 pass each) of one library under different environment
# settings:  CFG=c3 bash profiles/pmc_env_ab.sh <tag> "<ENV=VAL ...>" "<ENV=VAL ...>" ...
# Output under gpurun_out/pmc_<tag>/e<i>/{fetch,write}; summarise with python profiles/pmc_summary.py <tag> <kernel>.
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
B="bench.py --config ${CFG:-c3} --no-cpu-baseline --steps 3 --warmup 1 --warmup-min-s 0 --no-stats"
i=0
for envs in "$@"; do
  i=$((i + 1))
  OUT=gpurun_out/pmc_$TAG/e$i
  mkdir -p "$OUT"
  echo "$envs" > "$OUT/env.txt"
  (
    export $envs
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- python3 $B > "$OUT/fetch.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- python3 $B > "$OUT/write.log" 2>&1
  )
done
echo done
