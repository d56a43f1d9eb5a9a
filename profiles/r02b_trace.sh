#!/bin/bash
# kernel traces: rank 0's share of an 8-rank C3 frame, C2, C3 (per-frame timelines: profiles/timeline.py)
set -o pipefail
mkdir -p gpurun_out/r02h
export TMPDIR=/tmp
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02h/rank8 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stats > gpurun_out/r02h/rank8.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02h/c2 -o run -- python3 bench.py --config c2 --steps 30 --warmup 5 --no-cpu-baseline --no-stats > gpurun_out/r02h/c2.log 2>&1 || exit 2
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02h/c3 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stats > gpurun_out/r02h/c3.log 2>&1 || exit 3
echo ok
