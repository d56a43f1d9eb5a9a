#!/bin/bash
# Round-4 HEAD evidence on one MI355X (from the repo root): bash profiles/r04/refresh.sh <tag> [a|b]
# (part a: tests, bench lines, shares; part b: BVH timings, traces, rocprof stats + PMC; default both)
#  - the -m gpu suite (with the float64 COR report)
#  - bench lines: C3 at 100/20 with the CPU baseline, C3 driver-style 20/5, C2, C4, C5, C1
#  - every rank's 8-rank C3 and C4 share through the loopback exchange path, rank 0 of the 4- and 2-rank C3 shares
#  - BVH timings, kernel traces (C3 8-rank share, C2), rocprof stats + PMC passes of C3 (profiles/collect.sh)
# Each step has its own time limit; the first failure ends the script.
set -eo pipefail
TAG=${1:-r04}
PART=${2:-ab}
O=gpurun_out/$TAG
mkdir -p $O
if [[ $PART == *a* ]]; then
COR_F64_REPORT=$O/cor_f64_report.jsonl timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 400 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3_driver.json 2> $O/bench_c3_driver.err
for c in c2 c4 c5 c1; do timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err; done
echo benches done
bash profiles/r04/shares.sh $TAG c3 8 0 1 2 3 4 5 6 7 > $O/shares_c3r8.txt
bash profiles/r04/shares.sh $TAG c4 8 0 1 2 3 4 5 6 7 > $O/shares_c4r8.txt
bash profiles/r04/shares.sh $TAG c3 4 0 1 2 3 > $O/shares_c3r4.txt
bash profiles/r04/shares.sh $TAG c3 2 0 1 > $O/shares_c3r2.txt
echo shares done
fi
[[ $PART == *b* ]] || exit 0
timeout -k 10 200 python3 profiles/bvh_timing.py > $O/bvh.txt 2>&1
export TMPDIR=/tmp
GSRT_DEBUG_RANK_OF=8:4 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_c3r8 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stats > $O/tr_c3r8.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_c2 -o run -- python3 bench.py --config c2 --steps 30 --warmup 5 --no-cpu-baseline --no-stats > $O/tr_c2.log 2>&1
bash profiles/collect.sh $TAG c3
echo refreshed
