# finer render units for the share deal: kRun/16 (16 tiles) and kRun/8 (32 tiles) against kRun/4 (64 tiles, product)
set -o pipefail
cp 3dgs-raytrace_amd/gsrt/libgsrt_xd16.so 3dgs-raytrace_amd/gsrt/libgsrt_ab.so && \
bash profiles/r06/ab.sh r06_ab25_d16 c3:8:1 c3:8:2 c3:8:6 c4:8:6 c3:4:1 && \
cp 3dgs-raytrace_amd/gsrt/libgsrt_xd8.so 3dgs-raytrace_amd/gsrt/libgsrt_ab.so && \
bash profiles/r06/ab.sh r06_ab25_d8 c3:8:1 c3:8:2 c3:8:6 c4:8:6 c3:4:1
