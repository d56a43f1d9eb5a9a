#!/bin/bash
# diagnostic-build wave-cycle splits (C3, 8-rank C3 root share) and standalone kernel times of 8-rank C3 shares
set -eo pipefail
O=gpurun_out/r04diag
mkdir -p $O
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 120 python3 profiles/diag_split.py c3 > $O/diag_c3.txt 2>&1
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 python3 profiles/diag_split.py c3 > $O/diag_c3r8.txt 2>&1
export TMPDIR=/tmp
for r in 0 4; do
  GSRT_DEBUG_RANK_OF=8:$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/alone_r$r -o run -- python3 profiles/alone.py c3 40 > $O/alone_r$r.log 2>&1
done
echo ok
