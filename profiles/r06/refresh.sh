#!/bin/bash
# Round-6 end-of-round evidence on one MI355X (from the repo root): bash profiles/r06/refresh.sh <tag> [t][a][b][c]
#  t: the -m gpu suite (float64 COR report)
#  a: bench lines C3 (100/20 + CPU baseline), C3 driver-style 20/5, C2, C4, C5, C1
#  b: every rank's share through the loopback exchange path: 8-rank C3, C4 and C5, 4- and 2-rank C3 and C5
#  c: per config the bench under rocprofv3 --kernel-trace --stats, BVH timings, PMC passes of C3 and C5
# Each step has its own time limit; the first failure ends the script.
set -eo pipefail
TAG=${1:-r06}
PART=${2:-tabc}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [[ $PART == *t* ]]; then
COR_F64_REPORT=$O/cor_f64_report.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
fi
if [[ $PART == *a* ]]; then
timeout -k 10 400 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3_driver.json 2> $O/bench_c3_driver.err
for c in c2 c4 c5 c1; do timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err; done
echo benches done
fi
if [[ $PART == *b* ]]; then
bash profiles/r05/shares.sh $TAG c3 8 0 1 2 3 4 5 6 7 > $O/shares_c3r8.txt
bash profiles/r05/shares.sh $TAG c4 8 0 1 2 3 4 5 6 7 > $O/shares_c4r8.txt
bash profiles/r05/shares.sh $TAG c5 8 0 1 2 3 4 5 6 7 > $O/shares_c5r8.txt
bash profiles/r05/shares.sh $TAG c3 4 0 1 2 3 > $O/shares_c3r4.txt
bash profiles/r05/shares.sh $TAG c5 4 0 1 2 3 > $O/shares_c5r4.txt
bash profiles/r05/shares.sh $TAG c3 2 0 1 > $O/shares_c3r2.txt
bash profiles/r05/shares.sh $TAG c5 2 0 1 > $O/shares_c5r2.txt
echo shares done
fi
if [[ $PART == *c* ]]; then
for c in c3 c2 c4 c5 c1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kst_$c -o run -- python3 bench.py --config $c \
    --no-cpu-baseline --steps 50 --warmup 10 > $O/kst_$c.json 2> $O/kst_$c.err
done
timeout -k 10 200 python3 profiles/bvh_timing.py > $O/bvh.txt 2>&1
bash profiles/collect.sh $TAG c3
bash profiles/collect.sh ${TAG}_c5 c5
echo refreshed
fi
