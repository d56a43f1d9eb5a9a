#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of the bench workload for several builds:
#   bash profiles/kstats.sh <config> <lib names...>   -> gpurun_out/kstats_<lib>/run_kernel_stats.csv
set -e
CFG=$1; shift
export TMPDIR=/tmp
for lib in "$@"; do
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/kstats_$lib -o run -- python3 bench.py --config $CFG --no-cpu-baseline --no-stats --steps 20 --warmup 3 \
    > gpurun_out/kstats_$lib.log 2>&1
done
