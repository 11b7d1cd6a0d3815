"""bench.py's --gpus handling (CPU): a mismatched WORLD_SIZE is refused, an RCCL run with too
few visible GPUs is refused before any rank starts, and without a launcher --gpus N starts N
ranks through a torch.distributed.run child (never an exec) whose exit code it returns."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PCS_DIST_BACKEND"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True,
                          timeout=300)


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_rccl_refuses_more_gpus_than_visible():
    # no visible GPU (hidden even on a GPU machine): --gpus 8 must exit non-zero instead of
    # starting 8 ranks or timing one device
    r = _run(["--gpus", "8"], HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    assert r.returncode == 2
    assert "needs 8 visible GPUs" in r.stderr


def test_launcher_starts_n_ranks_as_child(monkeypatch):
    sys.path.insert(0, REPO)
    import bench
    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd: calls.append(cmd) or 7)
    monkeypatch.setenv("PCS_DIST_BACKEND", "gloo")
    monkeypatch.setattr(sys, "argv", [BENCH, "--gpus", "4", "--steps", "2"])
    assert bench.launch_ranks(4) == 7
    cmd = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"]


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0
