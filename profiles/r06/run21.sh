# the whole -m gpu suite at HEAD (after reverting the slot-stream three-slot variant)
set -o pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t21.log 2>&1
rc=$?
tail -3 gpurun_out/r06_t21.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t21.log | head -5; exit 1; fi
