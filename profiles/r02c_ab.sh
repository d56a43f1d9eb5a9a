#!/bin/bash
# One candidate change on one MI355X: GPU parity of the render/config tests on the product library, the A/B of
# a baseline library against it (C3, C2, 8-rank C3/C4 shares, two interleaved rounds), and a kernel trace of the
# product's 8-rank C3 share (profiles/timeline.py).   bash profiles/r02c_ab.sh <baseline lib> <tag>
set -o pipefail
A=$1; T=${2:-ab}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_render_gpu.py tests/test_configs_gpu.py tests/test_bvh_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
bash profiles/r02b_ab_all.sh $A libgsrt > $O/ab.log 2>&1 || exit 2
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/c3r8 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stats > $O/c3r8.log 2>&1 || exit 3
echo ok
