# the traversals' depth cull only where groups overflow (samples >= 16 per tile pixel, or groups 32 px wide: product) against
# everywhere (libgsrt_ab.so: the previous commit)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -k "depth_cull or pipelined or c5" --timeout 200 --timeout-method thread > gpurun_out/r06_t33.log 2>&1
rc=$?
tail -2 gpurun_out/r06_t33.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t33.log | head -5; exit 1; fi
bash profiles/r06/ab.sh r06_ab33 c3 c3:8:2 c4:8:6 c2 c4 c5
