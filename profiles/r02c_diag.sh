#!/bin/bash
# diagnostic build counters (traversal steps / nodes / cycles of the group lists) for C3 and C2
set -o pipefail
mkdir -p gpurun_out/diag
for c in c3 c2; do
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 120 python profiles/diag_split.py $c > gpurun_out/diag/diag_$c.log 2>&1 || exit 1
done
echo ok
