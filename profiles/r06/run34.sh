# experiment (out of tree, libgsrt_ab.so): no per-tile lists, every tile starts in its group's list (k_render_cor's
# continuation path filters it); checked against the oracle on a GPU test subset first
set -o pipefail
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_ab.so timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py tests/test_configs_gpu.py -m gpu -x -q -k "oracle or c3 or c2 or pipelined or c5" --timeout 200 --timeout-method thread > gpurun_out/r06_t34.log 2>&1
rc=$?
tail -2 gpurun_out/r06_t34.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t34.log | head -5; exit 1; fi
bash profiles/r06/ab.sh r06_ab34 c3 c2 c4 c5 c3:8:2
