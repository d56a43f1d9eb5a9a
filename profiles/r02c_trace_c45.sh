#!/bin/bash
# kernel traces of the C5 (dynamic: update + refit per frame) and C4 benches at HEAD (profiles/timeline.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02c_tr45
mkdir -p $O
for c in c5 c4; do
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-stats > $O/$c.log 2>&1 || exit 1
done
echo ok
