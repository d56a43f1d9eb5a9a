#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02f
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 120 python profiles/diag_split.py c3 > gpurun_out/r02f/diag_c3.log 2>&1 || exit 1
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so timeout -k 10 120 python profiles/diag_split.py c2 > gpurun_out/r02f/diag_c2.log 2>&1 || exit 2
timeout -k 10 300 bash profiles/rank_share.sh c3 > gpurun_out/r02f/rank_share.log 2>&1 || exit 3
timeout -k 10 400 bash profiles/ab.sh c3 libgsrt_xbase libgsrt_x2 libgsrt_xnew > gpurun_out/r02f/ab.log 2>&1 || exit 4
timeout -k 10 200 bash profiles/ab.sh c2 libgsrt_xbase libgsrt_xnew > gpurun_out/r02f/ab_c2.log 2>&1 || exit 5
echo ok
