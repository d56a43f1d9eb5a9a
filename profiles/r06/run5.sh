set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t5.log 2>&1
rc=$?
tail -3 gpurun_out/r06_t5.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t5.log | head -5; exit 1; fi
bash profiles/r06/ab.sh r06_ab5 c3 c3:8:2 c5:8:3 c5:8:3+GSRT_DEBUG_GROUP_TILES=2 c5 c4
