#!/bin/bash
# first-frames diagnostic: per-frame times of a fresh process, plain and after 300 ms of GPU matmuls
set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 120 python profiles/warmup_curve.py 60 > gpurun_out/r02b/warm.log 2>&1 || exit 1
timeout -k 10 120 python profiles/warmup_curve.py 60 0 300 > gpurun_out/r02b/warm_heat.log 2>&1 || exit 2
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02b/bench_20_5.log 2>&1 || exit 3
echo ok
