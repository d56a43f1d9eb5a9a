#!/bin/bash
# first GPU pass over the band partition: the -m gpu suite, 8-rank C3 shares, C3/C2 kernel stats against HEAD
set -eo pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/r05/shares.sh r05 c3 8 0 3 7
bash profiles/r05/kst.sh "c3 c2" libgsrt_xhead libgsrt_xn0 libgsrt
