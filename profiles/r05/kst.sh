#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of the bench workload, per config and build:
#   bash profiles/r05/kst.sh "<configs>" <lib names...>  -> gpurun_out/r05/kst_<cfg>_<lib>/run_kernel_stats.csv
set -eo pipefail
CFGS=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
for c in $CFGS; do for lib in "$@"; do
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/r05/kst_${c}_$lib -o run -- python3 bench.py --config $c --no-cpu-baseline --no-stats --steps 30 --warmup 5 \
    > gpurun_out/r05/kst_${c}_$lib.log 2>&1
  echo "$c $lib: $(grep -o '"value": [0-9.]*' gpurun_out/r05/kst_${c}_$lib.log)"
done; done
