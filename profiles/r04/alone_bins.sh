#!/bin/bash
# standalone kernel times (frames one at a time, rocprofv3 --kernel-trace --stats) with GSRT_BINS=1 and 0, C2 and C3
set -eo pipefail
export TMPDIR=/tmp
for v in 1 0; do
  for c in c2 c3; do
    GSRT_BINS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/alone_bins/${c}_$v -o run -- python3 profiles/alone.py $c 30 > gpurun_out/alone_bins_${c}_$v.log 2>&1
    echo "== $c GSRT_BINS=$v"
    python3 - "$c" "$v" <<'PY'
import csv, glob, sys
c, v = sys.argv[1], sys.argv[2]
f = sorted(glob.glob(f"gpurun_out/alone_bins/{c}_{v}/**/run_kernel_stats.csv", recursive=True))[-1]
for r in csv.DictReader(open(f)):
    if int(r["Calls"]) >= 20:
        print(f'  {r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
  done
done
