"""The multi-rank exchange on the HIP engine, several ranks on the box's one GPU.

RCCL refuses a communicator whose ranks share a device ("Duplicate GPU detected"), so
these runs use gloo: distributed.py stages the device tensors through host memory and
everything else — HipEngine's route / window / owner / pack / combine kernels, the
sync-free and synced exchanges, the overflow replays, the gather export, per-rank
write_redis, both replicated insert forms and bench.py's N > 1 step — is the code the
RCCL runs execute.  Results are checked against the single-filter oracle
(tests/dist_worker.py).  Times from these runs are not performance numbers.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def torchrun(world, script, args=(), env_extra=None, timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script, *args]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)


@pytest.mark.timeout(300)
# (the 10k, north-star x 8 and 200B x 8 runs are the poisoned test's: the same worker with
# every exchange buffer poisoned, a strictly stronger check; shards past 2^32 bits, nh > 1, run
# in the 200B x 8 poisoned case and the 200B x 2 uneven-batch case)
@pytest.mark.parametrize("world,m,k,block_log2", [
    (4, 9585058, 6, 12),            # 1M@1 %, four owners
    (3, 1437758757, 10, 20),        # 100M@0.1 %, odd shard count, 2^20-bit blocks
    (6, 3834023350947, 13, 20),     # P * nh = 18 windows: no chunk geometry, plain sync-free windows
])
def test_partitioned_hip_multirank(world, m, k, block_log2):
    cfg = {"m": m, "k": k, "block_log2": block_log2, "n": 800, "seed": 11, "engine": "hip"}
    if world == 6:
        cfg["chunks"] = False   # falls back to plain windows, no replays
    out = torchrun(world, os.path.join(HERE, "dist_worker.py"), env_extra={"BF_DIST_CFG": json.dumps(cfg)},
                   timeout=280)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,m,k,block_log2", [
    (2, 95851, 6, 10),              # 10k@1 %, small blocks: many blocks per shard
    (8, 9585058377, 6, 20),         # the north-star filter over eight owners
    (8, 3834023350947, 13, 20),     # BASELINE configs[4]: 200B@0.01 % partitioned x8 (nh = 2)
])
def test_partitioned_hip_multirank_poisoned(world, m, k, block_log2):
    """The same runs (forced overflows of the sync-free and synced exchanges included) with
    every window buffer poisoned before it is written: routed entries
    hold owner-local offset 1 (a bit the oracle leaves 0 at these sizes: a stray OR breaks
    the Redis string) and answer bytes 0 (a stray AND turns a member false)."""
    cfg = {"m": m, "k": k, "block_log2": block_log2, "n": 800, "seed": 11, "engine": "hip"}
    out = torchrun(world, os.path.join(HERE, "dist_worker.py"),
                   env_extra={"BF_DIST_CFG": json.dumps(cfg), "BFHIP_POISON_WINDOWS": "1"}, timeout=280)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,m,k,block_log2", [
    (3, 9585058, 6, 12),            # one rank brings an empty batch
    (2, 3834023350947, 13, 20),     # 200B at P = 2: shards past 2^32 bits, nh = 7 sub-range windows
])
def test_partitioned_hip_uneven_batches(world, m, k, block_log2):
    """Ranks bringing different batch sizes through the sync-free exchange, one
    rank past the agreed window bound (global overflow -> synced replay -> raised bound),
    and the pending-prefetch guards, on the HIP engine, windows poisoned."""
    cfg = {"case": "uneven", "m": m, "k": k, "block_log2": block_log2, "n": 300, "seed": 3, "engine": "hip"}
    out = torchrun(world, os.path.join(HERE, "dist_worker.py"),
                   env_extra={"BF_DIST_CFG": json.dumps(cfg), "BFHIP_POISON_WINDOWS": "1"}, timeout=280)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


@pytest.mark.parametrize("world", [2, 3])
def test_replicated_hip_multirank(world):
    cfg = {"case": "replicated", "m": 9585058, "k": 6, "n": 2000, "seed": 5, "engine": "hip"}
    out = torchrun(world, os.path.join(HERE, "dist_worker.py"), env_extra={"BF_DIST_CFG": json.dumps(cfg)},
                   timeout=110)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


@pytest.mark.timeout(300)
def test_replicated_hip_10b_x8():
    """BASELINE configs[3]: 10B@0.01 % (m = 191,701,167,547, k = 13, 6.98 GB reachable)
    replicated on 8 ranks, key batches sharded, through the digests insert and the pipelined
    sizes_start / gather_start / insert_gathered sequence bench.py --config 10b runs; every
    replica checked against the oracle (ruby.rb:57-63, compared by nonzero bytes)."""
    cfg = {"case": "replicated_big", "m": 191701167547, "k": 13, "n": 1500, "seed": 7, "engine": "hip"}
    out = torchrun(8, os.path.join(HERE, "dist_worker.py"), env_extra={"BF_DIST_CFG": json.dumps(cfg)},
                   timeout=280)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


@pytest.mark.timeout(300)
def test_replicated_bench_step_nstar_x2():
    """The exact step bench.py --gpus 2 times on the north-star filter (replicated, region
    sets, fused hash: distributed.ReplicatedPipeline), five steps with the wrap-around, every
    step's include? answers and both replicas' bitsets against the oracle; plus a damaged set
    buffer raising on every rank and one rank's oversized batch taking the digests form on
    every rank (tests/dist_worker.py rpipe_case).  The 10B x 8 run of the same step is in
    test_replicated_hip_10b_x8."""
    cfg = {"case": "rpipe", "m": 9585058377, "k": 6, "n": 60000, "steps": 5, "seed": 17, "engine": "hip"}
    out = torchrun(2, os.path.join(HERE, "dist_worker.py"), env_extra={"BF_DIST_CFG": json.dumps(cfg)},
                   timeout=280)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


def test_or_allreduce_device_tensors():
    cfg = {"case": "or_allreduce", "engine": "hip"}
    out = torchrun(3, os.path.join(HERE, "dist_worker.py"), env_extra={"BF_DIST_CFG": json.dumps(cfg)},
                   timeout=110)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,config,layout", [
    (4, "1m_big", "partitioned"),   # N >= 4 (auto)
    (2, "nstar", "replicated"),     # the north-star filter at N = 2 (auto: gather insert)
    (4, "nstar", "partitioned"),    # ... and at N = 4
    (2, "10b", "replicated"),       # BASELINE configs[3]'s layout: digests insert, 6.98 GB replicas
])
def test_bench_multirank_rehearsal(world, config, layout):
    """bench.py's N > 1 step, launched as the driver launches it (torch.distributed.run),
    with --dist-backend gloo: one JSON line from rank 0, the auto layout, every step's
    members found (bench.py asserts it on every rank)."""
    args = ["--gpus", str(world), "--config", config, "--steps", "2", "--warmup", "1", "--dist-backend", "gloo",
            "--no-secondary", "--no-cpu-baseline", "--no-host-api", "--no-reference-shapes"]
    out = torchrun(world, os.path.join(ROOT, "bench.py"), args, timeout=280)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["value"] > 0
    assert d["config"]["parallelism"].startswith(layout)
    assert "REHEARSAL" in d["config"]["parallelism"]


@pytest.mark.timeout(300)
def test_bench_plain_gpus_n_runs_n_ranks():
    """``python bench.py --gpus 2`` with no launcher around it: bench.py
    starts the two ranks itself and the line reports n_gpus == 2 from a 2-rank group (the
    driver's N = 2 layout on 1m_big: replicated, auto)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "1m_big", "--steps", "2",
            "--warmup", "1", "--dist-backend", "gloo", "--no-secondary", "--no-cpu-baseline", "--no-host-api",
            "--no-reference-shapes"]
    out = subprocess.run(args, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size_seen"] == 2 and d["value"] > 0
    assert d["launcher"].startswith("bench.py --gpus 2")
