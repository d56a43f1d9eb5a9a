# two-segment group lists (product build) against one segment (libgsrt_ab.so, -DGSRT_GROUP_SEGMENTS=1)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_render_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_t28.log 2>&1
rc=$?
tail -2 gpurun_out/r06_t28.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t28.log | head -5; exit 1; fi
bash profiles/r06/ab.sh r06_ab28 c5 c5:8:5 c5:8:1 c3 c4 c2
