#!/bin/bash
# kernel statistics of a rank share: alone (frames one at a time) and pipelined (bench.py), kernel trace + stats
#   bash profiles/r05/share_kst.sh <config> <N> <r>  -> gpurun_out/r05/kst_<cfg>_<N>_<r>_{alone,pipe}/
set -eo pipefail
CFG=$1; N=$2; R=$3
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
GSRT_DEBUG_RANK_OF=$N:$R timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kst_${CFG}_${N}_${R}_alone -o run -- python3 profiles/alone.py $CFG 40 > $O/kst_${CFG}_${N}_${R}_alone.log 2>&1
GSRT_DEBUG_RANK_OF=$N:$R timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kst_${CFG}_${N}_${R}_pipe -o run -- python3 bench.py --config $CFG --no-cpu-baseline --no-stats --steps 200 --warmup 20 > $O/kst_${CFG}_${N}_${R}_pipe.log 2>&1
for m in alone pipe; do
  echo "== $m"; python3 - "$O/kst_${CFG}_${N}_${R}_$m" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:12]:
    print(f"{r['Name'][:60]:60s} n={r['Calls']:>6s} avg={float(r['AverageNs'])/1e3:8.1f} us  tot%={float(r['Percentage']):5.1f}")
PY
done
