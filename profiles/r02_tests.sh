#!/bin/bash
# GPU parity suite (new config tests first), then driver-style and long bench runs
set -o pipefail
mkdir -p gpurun_out/r02d
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r02d/pytest_cfg.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02d/pytest.log 2>&1 || exit 2
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02d/bench_20_5.log 2>&1 || exit 3
timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r02d/bench_100_20.log 2>&1 || exit 4
echo ok
