#!/bin/bash
# interleaved A/B of environment settings on rank shares: bash profiles/r05/env_ab.sh <config> "<N:r ...>" "<env1>" "<env2>" ...
# (an env entry like "NCCL_MAX_NCHANNELS=2" or "-" for none)
set -eo pipefail
CFG=$1; SPECS=$2; shift 2
O=gpurun_out/r05_env; mkdir -p $O
for rep in 1 2; do
  for e in "$@"; do
    for spec in $SPECS; do
      tag=$(echo "$e" | tr -c 'A-Za-z0-9\n' '_')
      if [ "$e" = "-" ]; then envs=""; else envs="$e"; fi
      env $envs GSRT_DEBUG_RANK_OF=$spec timeout -k 10 150 python3 bench.py --config $CFG --no-cpu-baseline --no-stats \
        --steps 200 --warmup 20 > $O/${tag}_${spec/:/_}_$rep.json 2> $O/${tag}_${spec/:/_}_$rep.err
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d.get('rank_share_exchange_ms'))" \
        $O/${tag}_${spec/:/_}_$rep.json "$rep $e $CFG $spec"
    done
  done
done
