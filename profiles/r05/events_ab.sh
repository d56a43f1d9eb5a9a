#!/bin/bash
set -e
mkdir -p gpurun_out/evab
for r in 1 2 3; do
  for opt in "" "--no-events"; do
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-stats $opt > gpurun_out/evab/a_${r}_${opt:-ev}.json 2>/dev/null
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/evab/a_${r}_${opt:-ev}.json "100/20 r$r ${opt:-events}"
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-stats --steps 20 --warmup 5 $opt > gpurun_out/evab/b_${r}_${opt:-ev}.json 2>/dev/null
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/evab/b_${r}_${opt:-ev}.json "20/5 r$r ${opt:-events}"
  done
done
