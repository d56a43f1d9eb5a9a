#!/bin/bash
# round-2 first GPU call: parity at HEAD, driver-style and long bench, per-frame warmup curve
set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02a/bench_20_5.log 2>&1 || exit 2
timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r02a/bench_100_20.log 2>&1 || exit 3
timeout -k 10 120 python profiles/warmup_curve.py 60 > gpurun_out/r02a/warm.log 2>&1 || exit 4
timeout -k 10 120 python profiles/warmup_curve.py 60 2000 > gpurun_out/r02a/warm_idle.log 2>&1 || exit 5
echo ok
