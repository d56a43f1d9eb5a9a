#!/bin/bash
# A/B of experiment builds on several configs: bash profiles/r05/ab2.sh "<configs>" <libs...>
set -eo pipefail
CFGS=$1; shift
O=gpurun_out/r05; mkdir -p $O
for lib in "$@"; do
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 300 python3 -u -m pytest tests/test_render_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "cor_sh3 or cor_cloud_rgba or golden or c3_full_frame or tile_overflow or multipass or group_lists or stack_restart" \
    > $O/t_$lib.log 2>&1
  echo "$lib tests: $(tail -1 $O/t_$lib.log)"
done
for c in $CFGS; do bash profiles/ab.sh $c "$@" | sed "s/^/$c /"; done
