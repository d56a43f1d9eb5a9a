#!/bin/bash
# kernel traces at HEAD: rank 0's share of an 8-rank C3 frame, and one-GPU C2 (profiles/timeline.py reads them)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02c_tr
mkdir -p $O
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/c3r8 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stats > $O/c3r8.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/c2 -o run -- python3 bench.py --config c2 --steps 30 --warmup 5 --no-cpu-baseline --no-stats > $O/c2.log 2>&1 || exit 2
echo ok
