# attach (borrowed arrays) checks + C5 lines with attach and with copy
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_bvh_gpu.py -m gpu -x -v -k "attach or double_buffered or device_updates" --timeout 120 --timeout-method thread > gpurun_out/r06_t11.log 2>&1
rc=$?
tail -3 gpurun_out/r06_t11.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t11.log | head -5; exit 1; fi
bash profiles/r06/quick.sh r06_q11a c5 c5:8:3 c5:8:0 && \
BENCH_EXTRA="--update copy" bash profiles/r06/quick.sh r06_q11c c5 c5:8:3 c5:8:0
