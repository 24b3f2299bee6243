"""bench.py's entry point on the CPU (no GPU call is reached): `--gpus` is authoritative.

- Under a launcher (WORLD_SIZE set) every rank exits non-zero unless WORLD_SIZE == --gpus, so a mislabelled line
  cannot be printed.
- A bare `bench.py --gpus N` (N > 1, no WORLD_SIZE) is the launcher: it starts torch.distributed.run as a child.
  Here (no GPU) the RCCL form stops before that with a clear error naming the visible-GPU count; the GPU test
  `tests/test_gpu_dp.py::test_bench_py_bare_gpus2_spawns_ranks` runs the spawned ranks.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("world,gpus", [("2", "1"), ("1", "2"), ("4", "8")])
def test_world_size_must_equal_gpus(world, gpus):
    p = subprocess.run([sys.executable, BENCH, "--gpus", gpus, "--steps", "1"], env=_env(WORLD_SIZE=world),
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert f"WORLD_SIZE={world} but --gpus {gpus}" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bare_gpus_n_is_the_launcher_and_checks_devices():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--steps", "1"], env=_env(VQA_DIST_BACKEND="nccl"),
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "--gpus 8 needs 8 visible GPUs for RCCL" in p.stderr


def test_gpus_must_be_positive():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "0"], env=_env(), capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert p.returncode == 2 and "--gpus must be >= 1" in p.stderr


def test_launcher_command_shape(monkeypatch):
    """The child command: torch.distributed.run, one node, N processes per node, rendezvous on 127.0.0.1, this
    bench.py with the caller's own arguments; started with subprocess.call (a child, never an exec)."""
    sys.path.insert(0, ROOT)
    import importlib
    bench = importlib.import_module("bench")
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", [BENCH, "--gpus", "4", "--steps", "5"])
    monkeypatch.setenv("VQA_DIST_BACKEND", "gloo")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.main() == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert os.path.abspath(cmd[cmd.index("--master-port") + 2]) == os.path.abspath(BENCH)
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"]
    assert seen["env"]["MASTER_ADDR"] == "127.0.0.1"
