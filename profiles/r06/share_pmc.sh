#!/bin/bash
# verdict item 3: the 8-rank C3 share's render kernel against the whole frame's eighth.
#   1. wave timelines (diagnostic build with GSRT_WAVE_TIMES: per-workgroup start / end / CU of the last frame),
#   2. PMC passes of the same commands (kernels serialised: each kernel's own duration and counters)
#   bash profiles/r06/share_pmc.sh <tag> <spec>...      spec = whole | N:r
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for spec in "$@"; do
  if [ "$spec" = whole ]; then unset GSRT_DEBUG_RANK_OF; else export GSRT_DEBUG_RANK_OF=$spec; fi
  t=${spec//:/_}
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xwt.so timeout -k 10 120 python3 profiles/wave_times.py c3 > $O/wt_$t.txt 2> $O/wt_$t.err || exit 1
  B="bench.py --config c3 --no-cpu-baseline --no-stats --steps 20 --warmup 5 --warmup-min-s 0"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/sq_$t -o run -- python3 $B > $O/sq_$t.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/tcc_$t -o run -- python3 $B > $O/tcc_$t.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$t -o run -- python3 $B > $O/fetch_$t.log 2>&1 || exit 1
  echo "== $spec"; head -8 $O/wt_$t.txt
done
