#!/bin/bash
# diagnostic build: group-list phase split (traversal, cull+sort, group list write, tile tests, tile list output)
set -o pipefail
mkdir -p gpurun_out/diag2
for c in c4 c3 c2; do
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 150 python profiles/diag_split.py $c > gpurun_out/diag2/diag_$c.log 2>&1 || exit 1
done
echo ok
