#!/bin/bash
# C5 frames one at a time (update + refit + frame, then a synchronisation): each kernel's standalone duration
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_alone; mkdir -p $O
GSRT_DEBUG_RANK_OF=8:3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5r83 -o run -- python3 profiles/alone.py c5 40 > $O/c5r83.log 2>&1
head -14 $O/c5r83/run_kernel_stats.csv | cut -d, -f1-4
