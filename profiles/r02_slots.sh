#!/bin/bash
set -o pipefail
for lib in libgsrt_xr libgsrt_x3; do
  for n in 8 4; do
    GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so GSRT_DEBUG_RANK_OF=$n timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-stats > gpurun_out/slots_${lib}_$n.log 2>&1 || exit 2
    echo "$lib N=$n: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/slots_${lib}_$n.log | tr "\n" " ")"
  done
done
timeout -k 10 300 bash profiles/ab.sh c3 libgsrt_xr libgsrt_x3 || exit 3
timeout -k 10 300 bash profiles/ab.sh c2 libgsrt_xr libgsrt_x3 || exit 4
