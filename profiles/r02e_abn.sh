#!/bin/bash
# N-way A/B of library builds (GPU parity first on the product library), two interleaved rounds per config,
# then a kernel trace of each library on C2:
#   bash profiles/r02e_abn.sh <tag> "<lib> <lib> ..." <config[:ranks]>...
set -o pipefail
T=$1; LIBS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_bvh_gpu.py tests/test_configs_gpu.py tests/test_render_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for spec in "$@"; do
  cfg=${spec%%:*}; rk=${spec#*:}; [ "$rk" = "$spec" ] && rk=
  for r in 1 2; do for lib in $LIBS; do
    if [ -n "$rk" ]; then export GSRT_DEBUG_RANK_OF=$rk; else unset GSRT_DEBUG_RANK_OF; fi
    GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 150 python bench.py --config $cfg --no-cpu-baseline $BENCH_ARGS > $O/${cfg}_${rk}_${lib}_$r.log 2>&1 || exit 2
    echo "$cfg/${rk:-1} $lib r$r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $O/${cfg}_${rk}_${lib}_$r.log | tr "\n" " ")" >> $O/ab.log
  done; done
done
unset GSRT_DEBUG_RANK_OF
for lib in $LIBS; do
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$lib -o run -- python3 bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-stats > $O/trace_$lib.log 2>&1 || exit 3
done
echo ok
