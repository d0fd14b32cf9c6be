"""bench.py's multi-GPU layouts at world size 1 (RCCL communicator of one rank), as a child
process: the partitioned (route -> grouped send/recv -> owner ops -> packed answers ->
combine) and replicated (gather / OR-all-reduce insert) steps run end to end, every step's
members are found (bench.py asserts it), and the JSON line keeps the driver's contract."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mode,config", [("partitioned", "1m_big"), ("replicated", "1m_big"),
                                         ("partitioned", "nstar"), ("replicated", "nstar")])
def test_bench_layouts_world1(mode, config):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mode", mode, "--config", config, "--steps", "2",
           "--warmup", "1", "--no-secondary", "--no-cpu-baseline", "--no-host-api", "--no-reference-shapes"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    assert mode in d["config"]["parallelism"]
