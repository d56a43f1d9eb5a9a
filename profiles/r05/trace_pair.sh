#!/bin/bash
# kernel traces of one rank share for several builds: bash profiles/r05/trace_pair.sh <N:r> <libs...>
set -eo pipefail
SPEC=$1; shift
export TMPDIR=/tmp
O=gpurun_out/r05_tr; mkdir -p $O
for lib in "$@"; do
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so GSRT_DEBUG_RANK_OF=$SPEC timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $O/$lib -o run -- python3 bench.py --no-cpu-baseline --no-stats --steps 200 --warmup 20 \
    > $O/$lib.json 2> $O/$lib.err
  echo "$lib: $(grep -o '"ms_per_step": [0-9.]*' $O/$lib.json)"
done
