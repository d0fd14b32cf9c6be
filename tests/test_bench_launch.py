"""bench.py --gpus N launches N ranks or fails, checked on the CPU.

``--launch-check`` builds the process group exactly as a bench run does (gloo here, no GPU
work) and has rank 0 report the world it saw; the driver's own launch form
(torch.distributed.run) and the plain ``python bench.py --gpus N`` form must both give
n_gpus == N, and a launcher whose WORLD_SIZE differs from --gpus must fail.
"""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", **(env_extra or {}))
    return subprocess.run([sys.executable, *args], env=env, capture_output=True, text=True, timeout=timeout,
                          cwd=ROOT)


def _line(out):
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, (out.stdout[-2000:], out.stderr[-2000:])
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 3])
def test_plain_gpus_n_spawns_n_ranks(world):
    out = _run([BENCH, "--gpus", str(world), "--dist-backend", "gloo", "--launch-check"])
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_gpus"] == world and d["world_size_seen"] == world and d["self_launched"]


def test_torchrun_launch_form():
    from test_gpu_dist_gloo import free_port
    out = _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                "--master-port", str(free_port()), BENCH, "--gpus", "2", "--dist-backend", "gloo", "--launch-check"])
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_gpus"] == 2 and d["world_size_seen"] == 2 and not d["self_launched"]


def test_world_size_mismatch_fails():
    out = _run([BENCH, "--gpus", "2", "--launch-check"], env_extra={"WORLD_SIZE": "3", "RANK": "0"})
    assert out.returncode != 0
    assert "WORLD_SIZE=3" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]


def test_single_gpu_default_is_one_rank():
    out = _run([BENCH, "--launch-check", "--dist-backend", "gloo"])
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_gpus"] == 1 and d["world_size_seen"] == 1 and not d["self_launched"]
