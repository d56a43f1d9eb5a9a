#!/bin/bash
# Round-2 HEAD refresh on one MI355X: full GPU parity suite, driver-style bench of every config, then the
# rocprof kernel-trace + PMC profile of C3 (profiles/collect.sh) summarised by parse_pmc.py
set -o pipefail
O=gpurun_out/${1:-r02c}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || exit 2
for c in c2 c4 c5 c1; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit 3
done
timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c3_100.log 2>&1 || exit 4
bash profiles/collect.sh ${1:-r02c} c3 || exit 5
echo ok
