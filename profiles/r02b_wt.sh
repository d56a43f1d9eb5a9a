set -o pipefail
mkdir -p gpurun_out/wt
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xwt.so timeout -k 10 120 python profiles/wave_times.py c3 > gpurun_out/wt/c3.txt 2>&1 || exit 1
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xwt.so timeout -k 10 120 python profiles/wave_times.py c2 > gpurun_out/wt/c2.txt 2>&1 || exit 2
bash profiles/r02b_pmc_ab.sh ab1 libgsrt_xbase libgsrt_xC
