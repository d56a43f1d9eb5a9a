# all eight C5 rank shares with three slots, a trace of rank 5, C5 1-GPU A/B again
set -o pipefail
bash profiles/r06/quick.sh r06_q14 c5:8:0 c5:8:1 c5:8:2 c5:8:3 c5:8:4 c5:8:5 c5:8:6 c5:8:7 && \
bash profiles/r06/c5_shares.sh r06_s14 8 5 && \
python3 profiles/frame_timeline.py gpurun_out/r06_s14/trace_c5_8_5/run_kernel_trace.csv 60 2 && \
AB_ENV=GSRT_DEBUG_SLOTS=2 bash profiles/r06/ab.sh r06_ab14 c5 c5:4:1 c5:2:0
