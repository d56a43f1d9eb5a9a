#!/bin/bash
# Persistent render kernel diagnostics (needs profiles/experiments/persistent_render.diff applied: the GSRT_PERSIST and
# GSRT_PERSIST_Q knobs are not in HEAD): timing with per-XCD / single queues, and one
# FETCH_SIZE and one SQ pass against the one-tile kernel (C3, rocprofv3 --pmc with --kernel-trace only).
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/persist_diag
mkdir -p $O
bash profiles/r04/env_shares_ab.sh c3 1 0 "GSRT_PERSIST=0" "GSRT_PERSIST=5" "GSRT_PERSIST=5 GSRT_PERSIST_Q=1"
for v in 0 5; do
  GSRT_PERSIST=$v timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$v -o run -- python3 bench.py --no-cpu-baseline --no-stats --steps 3 --warmup 1 --warmup-min-s 0 > $O/fetch_$v.log 2>&1
  GSRT_PERSIST=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/sq_$v -o run -- python3 bench.py --no-cpu-baseline --no-stats --steps 3 --warmup 1 --warmup-min-s 0 > $O/sq_$v.log 2>&1
done
echo ok
