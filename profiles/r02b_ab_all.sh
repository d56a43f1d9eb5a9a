#!/bin/bash
# A/B of two library builds on C3, C2 and the 8-rank C3/C4 shares, two interleaved rounds each
#   bash profiles/r02b_ab_all.sh <libA> <libB>
set -o pipefail
A=$1; B=$2
mkdir -p gpurun_out/aball
for spec in "c3:" "c2:" "c3:8" "c4:8"; do
  cfg=${spec%%:*}; rk=${spec##*:}
  for r in 1 2; do for lib in $A $B; do
    if [ -n "$rk" ]; then export GSRT_DEBUG_RANK_OF=$rk; else unset GSRT_DEBUG_RANK_OF; fi
    GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/aball/${cfg}_${rk}_${lib}_$r.log 2>&1 || exit 1
    echo "$cfg/${rk:-1} $lib r$r: $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frame_ms_events": [0-9.]*' gpurun_out/aball/${cfg}_${rk}_${lib}_$r.log | tr "\n" " ")"
  done; done
done
