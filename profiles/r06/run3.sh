set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t2.log 2>&1
rc=$?
tail -3 gpurun_out/r06_t2.log
if [ $rc -ne 0 ] && grep -q -E "Fatal|fault|Aborted|core dumped|Segmentation" gpurun_out/r06_t2.log; then echo "GPU fault: stop"; exit 1; fi
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 120 python3 profiles/diag_split.py c5 > gpurun_out/r06_diag_c5.txt 2>&1 || exit 1
GSRT_DEBUG_RANK_OF=8:3 GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 120 python3 profiles/diag_split.py c5 > gpurun_out/r06_diag_c5r83.txt 2>&1 || exit 1
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 120 python3 profiles/diag_split.py c3 > gpurun_out/r06_diag_c3.txt 2>&1 || exit 1
cat gpurun_out/r06_diag_c5.txt gpurun_out/r06_diag_c5r83.txt gpurun_out/r06_diag_c3.txt
bash profiles/r06/c5_shares.sh r06_c5band 8 3 0 3 7
