#!/bin/bash
# HEAD check on one MI355X: full GPU parity suite, driver-style bench (C3), C2 bench
set -o pipefail
O=gpurun_out/${1:-r02b}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || exit 3
timeout -k 10 120 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2.log 2>&1 || exit 4
echo ok
