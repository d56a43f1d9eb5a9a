#!/bin/bash
# kernel traces at HEAD (profiles/timeline.py reads them): rank 0's share of 8-rank C3 and C4 frames, one-GPU C2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03}_tr
mkdir -p $O
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/c3r8 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stats > $O/c3r8.log 2>&1 || exit 1
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/c4r8 -o run -- python3 bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-stats > $O/c4r8.log 2>&1 || exit 2
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/c2 -o run -- python3 bench.py --config c2 --steps 30 --warmup 5 --no-cpu-baseline --no-stats > $O/c2.log 2>&1 || exit 3
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 python3 profiles/diag_split.py c3 > $O/diag_c3r8.txt 2>&1 || exit 4
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 120 python3 profiles/diag_split.py c3 > $O/diag_c3.txt 2>&1 || exit 5
echo ok
