# C5: 2x2-tile groups (GSRT_DEBUG_GROUP_TILES=2) against the default 4x4 (product), and the share wave timeline of
# rank 1 with the cost-ordered deal
set -o pipefail
AB_ENV=GSRT_DEBUG_GROUP_TILES=2 bash profiles/r06/ab.sh r06_ab18 c5 c5:8:5 c5:8:0 c5:4:1 && \
GSRT_DEBUG_RANK_OF=8:1 GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xwt.so timeout -k 10 120 python3 profiles/wave_times.py c3 > gpurun_out/r06_wt18_8_1.txt 2>&1 && \
GSRT_DEBUG_DEAL=0 GSRT_DEBUG_RANK_OF=8:1 GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xwt.so timeout -k 10 120 python3 profiles/wave_times.py c3 > gpurun_out/r06_wt18_8_1_centre.txt 2>&1
grep -A8 "k_render_cor" gpurun_out/r06_wt18_8_1.txt gpurun_out/r06_wt18_8_1_centre.txt
