# kernel timelines of the 1-GPU C2 and C4 frames (slot streams) and the 8-rank C3 share (rank 2)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_tr19; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --config c2 --steps 60 --warmup 10 --no-cpu-baseline --no-stats > $O/c2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 bench.py --config c4 --steps 60 --warmup 10 --no-cpu-baseline --no-stats > $O/c4.log 2>&1 || exit 2
GSRT_DEBUG_RANK_OF=8:2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3r82 -o run -- python3 bench.py --config c3 --steps 60 --warmup 10 --no-cpu-baseline --no-stats > $O/c3r82.log 2>&1 || exit 3
for c in c2 c4 c3r82; do echo "=== $c"; python3 profiles/frame_timeline.py $O/$c/run_kernel_trace.csv 50 2; done
