set -o pipefail
timeout -k 5 120 ./profiles/probes/copy_probe
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t9.log 2>&1
rc=$?
tail -3 gpurun_out/r06_t9.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t9.log | head -5; exit 1; fi
bash profiles/r06/alone_c5.sh > /dev/null 2>&1 && python3 profiles/frame_timeline.py gpurun_out/r06_alone/c5r83/run_kernel_trace.csv 30 1
bash profiles/r06/quick.sh r06_q9 c5 c5:8:3 c3
