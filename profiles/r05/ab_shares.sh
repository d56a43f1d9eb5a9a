#!/bin/bash
# interleaved A/B of rank shares and the 1-GPU line: bash profiles/r05/ab_shares.sh <config> "<N:r ...>" <libs...>
set -eo pipefail
CFG=$1; SPECS=$2; shift 2
O=gpurun_out/r05_ab; mkdir -p $O
for rep in 1 2; do
  for lib in "$@"; do
    for spec in $SPECS; do
      if [ "$spec" = "1" ]; then env_rank=""; else env_rank="GSRT_DEBUG_RANK_OF=$spec"; fi
      env $env_rank GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 150 python3 bench.py --config $CFG --no-cpu-baseline \
        --no-stats --steps 200 --warmup 20 > $O/${lib}_${spec/:/_}_$rep.json 2> $O/${lib}_${spec/:/_}_$rep.err
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'])" \
        $O/${lib}_${spec/:/_}_$rep.json "$rep $lib $CFG $spec"
    done
  done
done
