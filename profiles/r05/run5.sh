#!/bin/bash
set -eo pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3_driver.json 2> $O/bench_c3_driver.err
python3 -c "import json; d=json.load(open('$O/bench_c3_driver.json')); print('C3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
