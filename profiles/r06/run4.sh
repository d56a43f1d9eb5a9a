set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t4.log 2>&1
rc=$?
tail -3 gpurun_out/r06_t4.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t4.log | head -5; fi
if [ $rc -ne 0 ] && grep -q -E "Fatal|fault|Aborted|core dumped|Segmentation|Memory access" gpurun_out/r06_t4.log; then echo "GPU fault: stop"; exit 1; fi
bash profiles/r06/c5_shares.sh r06_c5side 8 3 0 1 2 3 4 5 6 7 && bash profiles/r06/quick.sh r06_q4 c5 c3 c3:8:2
