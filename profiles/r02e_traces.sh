#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace) of several library builds on several configs, for profiles/timeline.py:
#   bash profiles/r02e_traces.sh <tag> "<lib> <lib> ..." <config>...
set -o pipefail
T=$1; LIBS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for c in "$@"; do for lib in $LIBS; do
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/${c}_$lib -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-stats > $O/trace_${c}_$lib.log 2>&1 || exit 3
done; done
echo ok
