#!/bin/bash
# GSRT_RENDER_SPLIT A/B (render kernel in K launches) on C3, C2 and the 8-rank C3 share; parity of the render tests
set -o pipefail
mkdir -p gpurun_out/split
GSRT_RENDER_SPLIT=3 timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/split/pytest.log 2>&1 || exit 1
for c in c3 c2; do
  bash profiles/r02b_env_ab.sh $c "GSRT_RENDER_SPLIT=1" "GSRT_RENDER_SPLIT=2" "GSRT_RENDER_SPLIT=4" >> gpurun_out/split/ab.log 2>&1 || exit 2
done
bash profiles/r02b_env_ab.sh c3 "GSRT_DEBUG_RANK_OF=8 GSRT_RENDER_SPLIT=1" "GSRT_DEBUG_RANK_OF=8 GSRT_RENDER_SPLIT=2" "GSRT_DEBUG_RANK_OF=8 GSRT_RENDER_SPLIT=3" >> gpurun_out/split/ab.log 2>&1 || exit 3
echo ok
