#!/bin/bash
# Profiles the bench workload on one MI355X (run on the GPU box from the repo root):
#   1. kernel trace + stats of bench.py (per-kernel durations)
#   2. separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) with --kernel-trace only (no sys/runtime trace)
# Output under gpurun_out/prof_<tag>/; profiles/parse_pmc.py summarises it into profiles/.
set -euo pipefail
TAG=${1:-r02}
CFG=${2:-c3}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --config $CFG --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $B > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- python3 $B --steps 3 --warmup 1 --warmup-min-s 0 --no-stats > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- python3 $B --steps 3 --warmup 1 --warmup-min-s 0 --no-stats > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq" -o run -- python3 $B --steps 3 --warmup 1 --warmup-min-s 0 --no-stats > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq2" -o run -- python3 $B --steps 3 --warmup 1 --warmup-min-s 0 --no-stats > "$OUT/sq2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/sq3" -o run -- python3 $B --steps 3 --warmup 1 --warmup-min-s 0 --no-stats > "$OUT/sq3.log" 2>&1
echo done
