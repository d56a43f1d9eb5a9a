#!/bin/bash
# parity suite, rank shares (projection culling on / off), C3 + C2 A/B against a baseline library
set -o pipefail
mkdir -p gpurun_out/r02i
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02i/pytest.log 2>&1 || { tail -30 gpurun_out/r02i/pytest.log; exit 1; }
tail -1 gpurun_out/r02i/pytest.log
for n in 2 4 8; do
  for pa in 0 1; do
    GSRT_DEBUG_PROJECT_ALL=$pa GSRT_DEBUG_RANK_OF=$n timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-stats > gpurun_out/r02i/rank_${n}_$pa.log 2>&1 || exit 2
    echo "N=$n project_all=$pa: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r02i/rank_${n}_$pa.log | tr "\n" " ")"
  done
done
timeout -k 10 300 bash profiles/ab.sh c3 libgsrt_x2 libgsrt_xr || exit 3
timeout -k 10 300 bash profiles/ab.sh c2 libgsrt_x2 libgsrt_xr || exit 4
