"""Kernel timeline of pipelined frames from a rocprofv3 --kernel-trace CSV (diagnostic):

  python profiles/frame_timeline.py <run_kernel_trace.csv> [first_frame] [frames]

for frames first..first+frames-1 (k_render_cor dispatches, default: the middle of the run), every kernel that starts
between the previous render's start and this render's end, relative to this render's start (us)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    m = re.search(r"(k_\w+|rccl\w+|nccl\w+|fillBuffer\w*|copyBuffer\w*)", r["Kernel_Name"])
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:24]))
ev.sort()
ren = [e for e in ev if e[2] == "k_render_cor"]
first = int(sys.argv[2]) if len(sys.argv) > 2 else len(ren) // 2
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 3
for i in range(max(1, first), min(len(ren), first + nf)):
    t0 = ren[i][0]
    print(f"--- frame {i}: render {(ren[i][1] - t0) / 1e3:.1f} us, period {(t0 - ren[i - 1][0]) / 1e3:.1f} us")
    for s, e, n in ev:
        if ren[i - 1][0] <= s <= ren[i][1]:
            print(f"   {n:24s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} ({(e - s) / 1e3:.1f})")
