"""Per-frame kernel timeline from a rocprofv3 --kernel-trace CSV (diagnostic):

  python profiles/timeline.py <run_kernel_trace.csv> [frames]

prints, for the last `frames` k_render_cor dispatches, each kernel's start / end relative to that render's start
(us), so the critical path of a pipelined frame (prep on its own streams beside the previous render) is visible."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ev = []
for r in rows:
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:30]))
ev.sort()
renders = [e for e in ev if e[2] == "k_render_cor"]
for i in range(max(1, len(renders) - nf), len(renders)):
    t0 = renders[i][0]
    prev = renders[i - 1]
    print(f"--- frame {i}: render {(renders[i][1] - t0) / 1e3:.1f} us, period {(t0 - prev[0]) / 1e3:.1f} us")
    for s, e, n in ev:
        if prev[0] - 50_000 <= s <= renders[i][1] and n != "k_render_cor" or (s, e, n) in (prev, renders[i]):
            print(f"  {n:18s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f}  ({(e - s) / 1e3:.1f})")
