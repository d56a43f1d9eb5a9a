"""Probe: two ranks sharing GPU 0 through gsrt's RCCL path (render_sharded with the comm-stream overlap).
Result on the 1-GPU box: RCCL refuses two ranks on one device (ncclCommInitRank: invalid usage), so the
N > 1 RCCL path is exercised only on multi-GPU nodes; one GPU covers it with render_sharded_emulated.
Compares rank 0's gathered frame with a single-device render. Run on the GPU box from the repo root."""
import os
import sys
import multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "3dgs-raytrace_amd"))


def worker(rank, n, uid_q, res_q):
    import numpy as np
    import gsrt
    ctx = gsrt.Context(0)
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 200000, 42, True)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    sc.build_bvh()
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, 4, 16)
    if rank == 0:
        uid = gsrt.comm_unique_id()
        for _ in range(n - 1):
            uid_q.put(uid)
    else:
        uid = uid_q.get()
    ctx.comm_init(uid, n, rank)
    for _ in range(5):  # several frames back to back: both packed buffers and the overlap get used
        sc.render_sharded_async(ubo, gsrt.MODE_COR)
    img = sc.render_sharded(ubo, gsrt.MODE_COR)
    if rank == 0:
        single, _ = sc.render(ubo, gsrt.MODE_COR)
        res_q.put(bool(img.tobytes() == single.tobytes()))
    ctx.synchronize()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctxm = mp.get_context("spawn")
    uid_q, res_q = ctxm.Queue(), ctxm.Queue()
    ps = [ctxm.Process(target=worker, args=(r, n, uid_q, res_q)) for r in range(n)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
    codes = [p.exitcode for p in ps]
    print("exit codes", codes)
    print("gathered frame equals single-device frame:", res_q.get(timeout=5) if all(c == 0 for c in codes) else None)
