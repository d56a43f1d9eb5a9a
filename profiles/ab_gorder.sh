mkdir -p gpurun_out
for round in 1 2; do
  for v in "xbase 0" "xbase 1" "xgs432 0" "xgs432 1"; do
    set -- $v
    GSRT_GROUP_ORDER=$2 GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_$1.so timeout -k 10 120 python3 bench.py --no-cpu-baseline > gpurun_out/abg_$1_$2_$round.log 2>&1 || exit 1
    echo "$1 order=$2 round $round: $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"frame_ms_events": [0-9.]*' gpurun_out/abg_$1_$2_$round.log | tr "\n" " ")"
  done
done
