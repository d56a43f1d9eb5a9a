"""Which of a gsrt context's streams share a hardware queue (after comm_init_loopback, as bench.py's rank shares run):
a spin kernel (torch.cuda._sleep, ~2 ms) on stream a, then a tiny kernel on stream b; b's wait shows a shared FIFO.

  python profiles/probes/gsrt_queue_map.py [pad]     pad: K idle default-priority streams created before the context
                                                      (another library's streams); GSRT_DEBUG_LAZY_STREAMS=1 for the
                                                      round-5 creation order"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "3dgs-raytrace_amd"))
import gsrt  # noqa: E402

pad = int(sys.argv[1]) if len(sys.argv) > 1 else 0
x = torch.zeros(16, device="cuda")
torch.cuda.synchronize()
extra = [torch.cuda.Stream() for _ in range(pad)]
ctx = gsrt.Context(0)
ctx.comm_init_loopback()
ctx.update_stream  # (created now when lazy)
st = {k: v for k, v in ctx.debug_streams.items() if v}
st["torch"] = torch.cuda.current_stream().cuda_stream
for i, e in enumerate(extra):
    st[f"pad{i}"] = e.cuda_stream
names = list(st)
print(f"lazy={os.environ.get('GSRT_DEBUG_LAZY_STREAMS', '0')} pad={pad}: ms for a tiny kernel on the column's stream "
      f"while the row's stream spins ~2 ms ('*' = shares a queue)")
print(" " * 10 + "".join(f"{n:>10s}" for n in names))
for a in names:
    row = []
    for b in names:
        if a == b:
            row.append("-")
            continue
        sa, sb = torch.cuda.ExternalStream(st[a]), torch.cuda.ExternalStream(st[b])
        with torch.cuda.stream(sa):
            torch.cuda._sleep(4_000_000)
        t0 = time.perf_counter()
        with torch.cuda.stream(sb):
            x.add_(1.0)
        sb.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize()
        row.append(f"{dt:.2f}{'*' if dt > 1.0 else ''}")
    print(f"{a:>10s}" + "".join(f"{v:>10s}" for v in row))
