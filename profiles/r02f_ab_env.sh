#!/bin/bash
# A/B of a runtime knob on the product library (extra bench flags in $BENCH_ARGS):
#   bash profiles/r02f_ab_env.sh <tag> <VAR> "<v1> <v2>" <config[:ranks]>...
set -o pipefail
T=$1; VAR=$2; VALS=$3; shift 3
O=gpurun_out/$T
mkdir -p $O
for spec in "$@"; do
  cfg=${spec%%:*}; rk=${spec#*:}; [ "$rk" = "$spec" ] && rk=
  for r in 1 2; do for v in $VALS; do
    if [ -n "$rk" ]; then export GSRT_DEBUG_RANK_OF=$rk; else unset GSRT_DEBUG_RANK_OF; fi
    env $VAR=$v timeout -k 10 150 python bench.py --config $cfg --no-cpu-baseline $BENCH_ARGS > $O/${cfg}_${rk}_${v}_$r.log 2>&1 || exit 2
    echo "$cfg/${rk:-1} $VAR=$v r$r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/${cfg}_${rk}_${v}_$r.log | tr "\n" " ")" >> $O/ab.log
  done; done
done
echo ok
