#!/bin/bash
set -eo pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_render_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "shard or group or c3_full or stack or overflow" > $O/gpu_tests2.log 2>&1 || { tail -40 $O/gpu_tests2.log; exit 1; }
tail -1 $O/gpu_tests2.log
bash profiles/r05/kst.sh "c3 c2" libgsrt_xhead libgsrt
bash profiles/r05/shares.sh r05 c3 8 0 3 7
