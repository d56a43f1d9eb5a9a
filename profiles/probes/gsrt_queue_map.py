"""Which of a gsrt context's streams share a hardware queue (after comm_init_loopback, as bench.py's rank shares run):
a spin kernel (torch.cuda._sleep) on stream a, then a tiny kernel on stream b; b's wait shows a shared FIFO.

  GSRT_LIB_PATH=... python profiles/probes/gsrt_queue_map.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "3dgs-raytrace_amd"))
import gsrt  # noqa: E402

ctx = gsrt.Context(0)
ctx.comm_init_loopback()
st = {"render": ctx.stream, "prep/slot0": ctx.prep_stream, "comm": ctx.comm_stream,
      "torch": torch.cuda.current_stream().cuda_stream}
x = torch.zeros(16, device="cuda")
torch.cuda.synchronize()
names = list(st)
print(os.path.basename(os.environ.get("GSRT_LIB_PATH", "libgsrt.so")))
print(" " * 12 + "".join(f"{n:>12s}" for n in names))
for a in names:
    row = []
    for b in names:
        if a == b:
            row.append("-")
            continue
        sa, sb = torch.cuda.ExternalStream(st[a]), torch.cuda.ExternalStream(st[b])
        with torch.cuda.stream(sa):
            torch.cuda._sleep(4_000_000)  # ~2 ms
        t0 = time.perf_counter()
        with torch.cuda.stream(sb):
            x.add_(1.0)
        sb.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize()
        row.append(f"{dt:.2f}ms")
    print(f"{a:>12s}" + "".join(f"{v:>12s}" for v in row))
