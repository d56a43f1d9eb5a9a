#!/bin/bash
# GPU parity suite on the product library, then A/B of experiment builds on C3 (and optional more configs)
#   bash profiles/r02_ab.sh <tag> <libA> <libB> [configs...]
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
CFGS=${@:-c3}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for c in $CFGS; do timeout -k 10 300 bash profiles/ab.sh $c $A $B || exit 2; done
