"""bench.py's multi-GPU launch contract (CPU only: every case here ends before a GPU call).

- `bench.py --gpus N` without WORLD_SIZE becomes N ranks: a child torch.distributed.run, started before any GPU
  call (no exec), rendezvous on 127.0.0.1;
- under a launcher, WORLD_SIZE must equal --gpus, else exit status 2 (an N-GPU line is never a 1-GPU measurement).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (numpy only at import time)


def run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=120)


def test_launch_command_shape():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "20", "--warmup", "5"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.abspath(BENCH))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]  # the same bench arguments, in order


def test_print_launch_without_world_size():
    r = run(["--gpus", "4", "--steps", "3", "--print-launch"])
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])
    assert "--nproc-per-node=4" in cmd
    assert cmd[cmd.index(os.path.abspath(BENCH)) + 1:] == ["--gpus", "4", "--steps", "3", "--print-launch"]
    port = int([a for a in cmd if a.startswith("--master-port=")][0].split("=")[1])
    assert 0 < port < 65536


@pytest.mark.parametrize("world,gpus", [("1", "8"), ("8", "1"), ("2", "4")])
def test_world_size_mismatch_exits_nonzero(world, gpus):
    r = run(["--gpus", gpus], {"WORLD_SIZE": world, "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert f"WORLD_SIZE={world}" in r.stderr and r.stdout == ""


def test_more_gpus_than_visible_exits_nonzero():
    # this container has no GPU: the child launch is refused before it starts (on the GPU box: 1 GPU < 2)
    import torch

    if torch.cuda.device_count() >= 64:
        pytest.skip("machine with 64+ GPUs")
    r = run(["--gpus", "64"])
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr, (r.returncode, r.stderr)


def test_zero_gpus_refused():
    r = run(["--gpus", "0"])
    assert r.returncode == 2


def test_warm_up_single_rank_counts():
    calls = {"frames": 0, "syncs": 0}
    t = [0.0]

    def frame():
        calls["frames"] += 1
        t[0] += 0.01  # 10 ms per frame

    def sync():
        calls["syncs"] += 1

    n = bench.warm_up(frame, sync, 5, 0.3, clock=lambda: t[0])
    assert n == calls["frames"] and n % bench.WARM_CHUNK == 0
    assert n >= 5 and n * 0.01 >= 0.3 and n - bench.WARM_CHUNK < 30  # stops at the first chunk past 0.3 s
    assert calls["syncs"] == n // bench.WARM_CHUNK


def _warm_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = [0.0]
    per_frame = 0.01 if rank == 0 else 0.002  # rank 1's clock says it is done much later

    def frame():
        t[0] += per_frame

    def agree(done):
        v = torch.tensor([1 if done else 0], dtype=torch.int64)
        dist.all_reduce(v, op=dist.ReduceOp.MIN)
        return bool(v[0])

    n = bench.warm_up(frame, lambda: None, 5, 0.3, agree, clock=lambda: t[0])
    q.put((rank, n))
    dist.destroy_process_group()


def test_warm_up_ranks_agree_gloo():
    """With N ranks every rank runs the same number of warm-up frames (the frames' gathers pair up), even when their
    own clocks would stop them at different chunks: the all-reduce waits for the slowest."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_warm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == res[1] == 152  # rank 1 needs 0.3 / 0.002 = 150 frames: 19 chunks of 8
