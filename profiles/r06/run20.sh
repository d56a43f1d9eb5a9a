# three slots on slot streams too (frames alternate streams; product) against two slots (GSRT_DEBUG_SLOTS=2)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_render_gpu.py tests/test_bvh_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_t20.log 2>&1
rc=$?
tail -2 gpurun_out/r06_t20.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t20.log | head -5; exit 1; fi
AB_ENV=GSRT_DEBUG_SLOTS=2 bash profiles/r06/ab.sh r06_ab20 c2 c4 c3 c3:8:2 c3:8:1 c4:8:6 c4:8:2 c3:4:1 c5:8:5
