#!/bin/bash
# GPU suite, then every rank's 8-rank C3 / C4 share (default deal)
set -eo pipefail
TAG=${1:-r04b}
mkdir -p gpurun_out/$TAG
COR_F64_REPORT=gpurun_out/$TAG/cor_f64_report.jsonl timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$TAG/gpu_tests.log
bash profiles/r04/shares.sh $TAG c3 8 0 1 2 3 4 5 6 7
bash profiles/r04/shares.sh $TAG c4 8 0 1 2 3 4 5 6 7
