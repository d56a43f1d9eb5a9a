#!/bin/bash
# Diagnostic (libgsrt_xskip, never the product): frame period when the prep kernels of static frames are skipped
# after frame 8 (GSRT_X_SKIP bits: 1 projection, 2 frontier, 4 group lists): what each costs the frame
set -o pipefail
O=gpurun_out/skip
mkdir -p $O
for spec in c3:8 c2: c4: c3:; do
  cfg=${spec%%:*}; rk=${spec##*:}
  for x in 0 1 2 4 7; do
    if [ -n "$rk" ]; then export GSRT_DEBUG_RANK_OF=$rk; else unset GSRT_DEBUG_RANK_OF; fi
    GSRT_X_SKIP=$x GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xskip.so timeout -k 10 150 python bench.py --config $cfg --no-cpu-baseline --no-stats > $O/${cfg}_${rk}_$x.log 2>&1 || exit 1
    echo "$cfg/${rk:-1} skip=$x: $(grep -o '"ms_per_step": [0-9.]*' $O/${cfg}_${rk}_$x.log)" >> $O/skip.log
  done
done
echo ok
