#!/bin/bash
# group lists at C4/C5: diagnostic counters (lengths, overflows, cycle split) and the 2x2 / 4x4 group-size A/B
set -o pipefail
O=gpurun_out/gl
mkdir -p $O
for c in c4 c5; do
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 150 python profiles/diag_split.py $c > $O/diag_$c.log 2>&1 || exit 1
done
bash profiles/r02b_env_ab.sh c4 "GSRT_GROUP_TILES=4" "GSRT_GROUP_TILES=2" > $O/ab_c4.log 2>&1 || exit 2
bash profiles/r02b_env_ab.sh c5 "GSRT_GROUP_TILES=4" "GSRT_GROUP_TILES=2" > $O/ab_c5.log 2>&1 || exit 3
echo ok
