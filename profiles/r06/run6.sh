set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t6.log 2>&1
rc=$?
tail -3 gpurun_out/r06_t6.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t6.log | head -5; exit 1; fi
bash profiles/r06/quick.sh r06_q6 c3 c5 c4 c2 c3:8:2 c5:8:0 c5:8:3 c5:8:7 && bash profiles/r06/c5_shares.sh r06_c5db 8 3
