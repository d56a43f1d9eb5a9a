# all eight C5 rank shares (attach), then a pipelined kernel trace of rank 3 and its frame timeline
set -o pipefail
bash profiles/r06/quick.sh r06_q12 c5:8:0 c5:8:1 c5:8:2 c5:8:3 c5:8:4 c5:8:5 c5:8:6 c5:8:7 && \
bash profiles/r06/c5_shares.sh r06_s12 8 3 && \
python3 profiles/frame_timeline.py gpurun_out/r06_s12/trace_c5_8_3/run_kernel_trace.csv 60 2 && \
head -16 gpurun_out/r06_s12/trace_c5_8_3/run_kernel_stats.csv | cut -d, -f1-4
