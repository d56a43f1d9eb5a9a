set -o pipefail
mkdir -p gpurun_out/wt
export GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xwt.so
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 python profiles/wave_times.py c3 > gpurun_out/wt/c3_rank8.txt 2>&1 || exit 1
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 python profiles/wave_times.py c4 > gpurun_out/wt/c4_rank8.txt 2>&1 || exit 2
unset GSRT_LIB_PATH
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/wt/bench_c3_rank8.log 2>&1 || exit 3
GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 python bench.py --config c4 --no-cpu-baseline > gpurun_out/wt/bench_c4_rank8.log 2>&1 || exit 4
