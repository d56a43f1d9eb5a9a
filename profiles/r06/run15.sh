# hardware-queue map and creation-order A/Bs (eager fixed order = product; lazy = round-5 order; padK = K idle
# default-priority streams created before the context)
set -o pipefail
mkdir -p gpurun_out/r06_q15
for v in "" "GSRT_DEBUG_LAZY_STREAMS=1"; do
  for pad in 0 1 2 3; do
    env $v timeout -k 10 60 python3 profiles/probes/gsrt_queue_map.py $pad >> gpurun_out/r06_q15/queue_map.txt 2>&1 || exit 1
  done
done
cat gpurun_out/r06_q15/queue_map.txt
for v in GSRT_DEBUG_LAZY_STREAMS=1 GSRT_BENCH_PAD_STREAMS=1 GSRT_BENCH_PAD_STREAMS=2 GSRT_BENCH_PAD_STREAMS=3; do
  echo "== ab: $v"
  AB_ENV=$v bash profiles/r06/ab.sh r06_ab15_${v##*=}${v%%_STREAMS*} c3:8:0 c3:8:1 c3:4:0 c3:2:1 c5:8:5 || exit 1
done
