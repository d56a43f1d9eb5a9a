#!/bin/bash
# interleaved A/B of the product library against gsrt/libgsrt_ab.so (make ab AB_FLAGS=...), or against the product
# library under the environment AB_ENV=VAR=V, two rounds:
#   bash profiles/r06/ab.sh <tag> <spec>...     spec = config[:N:r][+ENV=V]  (N:r = GSRT_DEBUG_RANK_OF rank share)
set -eo pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for round in 1 2; do
  for spec in "$@"; do
    base=${spec%%+*}; envs=""; [ "$spec" != "$base" ] && envs=${spec#*+}
    IFS=: read -r CFG N R <<< "$base"
    for lib in prod ab; do
      ( if [ -n "$N" ]; then export GSRT_DEBUG_RANK_OF=$N:$R; fi
        if [ -n "$envs" ]; then export ${envs//+/ }; fi
        if [ $lib = ab ]; then
          if [ -n "$AB_ENV" ]; then export $AB_ENV; else export GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_ab.so; fi
        fi
        f=$O/${spec//[:+=]/_}_${lib}_$round.json
        timeout -k 10 150 python3 bench.py --config $CFG --no-cpu-baseline --no-stats --steps 100 --warmup 20 > $f 2> ${f%.json}.err
        python3 -c "import json; d=json.load(open('$f')); print('$round $spec $lib', d['ms_per_step'], 'ms')" )
    done
  done
done
