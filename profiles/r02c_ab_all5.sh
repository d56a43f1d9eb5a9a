#!/bin/bash
# Full GPU parity suite on the product library, then the A/B of a baseline library against it on C3, C2, C4,
# C5 and the 8-rank C3/C4 shares (two interleaved rounds), and kernel traces of the product (C2, 8-rank C3).
#   bash profiles/r02c_ab_all5.sh <baseline lib> <tag>
set -o pipefail
A=$1; T=$2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for spec in c3: c2: c4: c5: c3:8 c4:8; do
  cfg=${spec%%:*}; rk=${spec##*:}
  for r in 1 2; do for lib in $A libgsrt; do
    if [ -n "$rk" ]; then export GSRT_DEBUG_RANK_OF=$rk; else unset GSRT_DEBUG_RANK_OF; fi
    GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 150 python bench.py --config $cfg --no-cpu-baseline > $O/${cfg}_${rk}_${lib}_$r.log 2>&1 || exit 2
    echo "$cfg/${rk:-1} $lib r$r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $O/${cfg}_${rk}_${lib}_$r.log | tr "\n" " ")" >> $O/ab.log
  done; done
done
unset GSRT_DEBUG_RANK_OF
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/c2 -o run -- python3 bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-stats > $O/trace_c2.log 2>&1 || exit 3
GSRT_DEBUG_RANK_OF=8 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/c3r8 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stats > $O/trace_c3r8.log 2>&1 || exit 4
echo ok
