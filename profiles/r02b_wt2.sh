set -o pipefail
mkdir -p gpurun_out/wt
export GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xwt.so
timeout -k 10 120 python profiles/wave_times.py c3 > gpurun_out/wt/c3b.txt 2>&1 || exit 1
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 python profiles/wave_times.py c3 > gpurun_out/wt/c3b_rank8.txt 2>&1 || exit 2
