#!/bin/bash
# per-dispatch effective clock (GRBM_GUI_ACTIVE / 8 / duration) over the first frames of a fresh process
set -o pipefail
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/r02c/clk -o run -- python3 profiles/warmup_curve.py 60 > gpurun_out/r02c/clk.log 2>&1 || exit 1
echo ok
