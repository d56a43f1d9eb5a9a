#!/bin/bash
# kernel traces of rank 0's share of an 8-rank C3 frame for library builds:  bash profiles/r02b_trace2.sh <libs...>
set -o pipefail
export TMPDIR=/tmp
for lib in "$@"; do
  mkdir -p gpurun_out/r02i/$lib
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02i/$lib -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stats > gpurun_out/r02i/$lib.log 2>&1 || exit 1
done
echo ok
