#!/bin/bash
# Round-5 A/B: SH-3 rows from SGPRs (scalar loads) against LDS broadcasts (GSRT_SH_SMEM 0-3) and HEAD.
# Parity subset per build first (any failure ends the script), then two interleaved C3 bench rounds.
set -eo pipefail
O=gpurun_out/r05; mkdir -p $O
for lib in "$@"; do
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 300 python3 -u -m pytest tests/test_render_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "cor_sh3 or cor_cloud_rgba or golden or c3_full_frame or tile_overflow or multipass" \
    > $O/t_$lib.log 2>&1
  echo "$lib tests: $(tail -1 $O/t_$lib.log)"
done
bash profiles/ab.sh c3 "$@"
