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
