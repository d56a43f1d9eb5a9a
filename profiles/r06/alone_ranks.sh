#!/bin/bash
# every 8-rank C3 share's kernels run one frame at a time (profiles/alone.py: synchronised after each frame, so each
# kernel runs without the neighbouring frames' beside it) under rocprofv3 --kernel-trace --stats; prints the render
# kernel's mean standalone duration per rank, and the whole frame's for reference.   bash profiles/r06/alone_ranks.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/whole -o run -- python3 profiles/alone.py c3 30 > $O/whole.log 2>&1 || exit 1
for r in 0 1 2 3 4 5 6 7; do
  GSRT_DEBUG_RANK_OF=8:$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r$r -o run -- python3 profiles/alone.py c3 40 > $O/r$r.log 2>&1 || exit 1
done
python3 - "$O" <<'PY'
import csv, sys, os
O = sys.argv[1]
def render(d):
    rows = [r for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))) if "k_render_cor" in r["Kernel_Name"]]
    t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    t = t[5:] if len(t) > 10 else t   # (the share runs three whole frames first; skip the first frames)
    t.sort()
    return len(t), sum(t) / len(t), t[len(t) // 2]
n, m, med = render(os.path.join(O, "whole"))
print(f"whole frame: render kernel mean {m:.1f} us, median {med:.1f} us over {n} frames (1/8: {m / 8:.1f} us)")
for r in range(8):
    n, m, med = render(os.path.join(O, f"r{r}"))
    print(f"8-rank C3 rank {r}: render kernel mean {m:.1f} us, median {med:.1f} us over {n} frames")
PY
