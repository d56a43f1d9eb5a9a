set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t10.log 2>&1
rc=$?
tail -3 gpurun_out/r06_t10.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t10.log | head -5; exit 1; fi
bash profiles/r06/alone_c5.sh > /dev/null 2>&1 && python3 profiles/frame_timeline.py gpurun_out/r06_alone/c5r83/run_kernel_trace.csv 30 1
bash profiles/r06/quick.sh r06_q10 c5 c5:8:3 c5:8:0
bash profiles/r06/ab.sh r06_ab10 c3:8:2 c3:8:5 c4:8:6 c4:8:1 c3
