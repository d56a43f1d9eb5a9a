#!/bin/bash
# persistent k_render_cor A/B (GSRT_PERSIST = waves per SIMD; 0 = one workgroup per tile) against the HEAD library
# before the change (libgsrt_xbase), two interleaved rounds each: C3, C2, and the 8-rank C3 share of rank 4
set -eo pipefail
B="GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xbase.so"
bash profiles/ab_env.sh c3 "$B" "GSRT_PERSIST=0" "GSRT_PERSIST=5" "GSRT_PERSIST=4"
bash profiles/ab_env.sh c2 "$B" "GSRT_PERSIST=0" "GSRT_PERSIST=5" "GSRT_PERSIST=4"
bash profiles/ab_env.sh c3 "GSRT_DEBUG_RANK_OF=8:4 $B" "GSRT_DEBUG_RANK_OF=8:4 GSRT_PERSIST=0" "GSRT_DEBUG_RANK_OF=8:4 GSRT_PERSIST=5" "GSRT_DEBUG_RANK_OF=8:4 GSRT_PERSIST=4" "GSRT_DEBUG_RANK_OF=8:4 GSRT_PERSIST=3"
