#!/bin/bash
# Round-end measurement refresh on one MI355X: bench lines for every config, BVH timings, rocprof profiles.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/bench_c3.log 2>&1
for c in c2 c4 c5; do timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1; done
timeout -k 10 200 python3 profiles/bvh_timing.py > gpurun_out/bvh.log 2>&1
bash profiles/collect.sh r01 c3
