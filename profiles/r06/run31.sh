# the group lists' depth cull only where tiles hold >= 16 samples per pixel (product) against everywhere (libgsrt_ab.so:
# the previous commit)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -k "depth_cull or pipelined or c5" --timeout 200 --timeout-method thread > gpurun_out/r06_t31.log 2>&1
rc=$?
tail -2 gpurun_out/r06_t31.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t31.log | head -5; exit 1; fi
bash profiles/r06/ab.sh r06_ab31 c3 c2 c4 c5 c5:8:5
