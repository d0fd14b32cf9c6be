"""Multi-process partitioned filter over gloo on the CPU (world size 2 and 3).

Checks redis-bloomfilter_amd/distributed.py's exchange (route -> all_to_all ->
owner op -> reverse all_to_all -> combine) and the block-cyclic Redis-string
assembly against a single-filter oracle run.  The GPU primitives behind the
same engine interface are checked in tests/test_gpu_distributed.py.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,m,k,block_log2", [
    (2, 95851, 6, 10),              # 10k@1%, small blocks: many blocks per shard
    (3, 9585058, 6, 12),            # 1M@1%, odd shard count
    (2, 191701167547, 13, 20),      # 10B@0.01%: reach-limited prefix, no modulo
])
def test_partitioned_gloo(world, m, k, block_log2):
    env = dict(os.environ)
    env["BF_DIST_CFG"] = json.dumps({"m": m, "k": k, "block_log2": block_log2, "n": 800, "seed": 11})
    env["BFHIP_STANDALONE"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(HERE, "dist_worker.py")]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


@pytest.mark.parametrize("world,m,k,block_log2", [
    (2, 95851, 6, 10),
    (3, 9585058, 6, 12),            # one rank brings an empty batch
])
def test_partitioned_uneven_batches_gloo(world, m, k, block_log2):
    """Ranks with different batch sizes through the sync-free exchange, a batch
    past the agreed window bound on one rank (global overflow -> synced replay), and the
    pending-prefetch guards."""
    env = dict(os.environ)
    env["BF_DIST_CFG"] = json.dumps({"case": "uneven", "m": m, "k": k, "block_log2": block_log2, "n": 300,
                                     "seed": 3})
    env["BFHIP_STANDALONE"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(HERE, "dist_worker.py")]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


@pytest.mark.parametrize("world", [2, 3])
def test_or_allreduce_gloo(world):
    """The replicated filter's OR-all-reduce (all_to_all + local OR + all_gather)."""
    env = dict(os.environ)
    env["BF_DIST_CFG"] = json.dumps({"case": "or_allreduce"})
    env["BFHIP_STANDALONE"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(HERE, "dist_worker.py")]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "DIST_RESULT ok" in out.stdout


def test_ownership_map_properties(pkg):
    D = pkg.distributed if hasattr(pkg, "distributed") else __import__("redis_bloomfilter_amd.distributed",
                                                                       fromlist=["x"])
    rng = np.random.default_rng(5)
    reach = 13 * 0xFFFFFFFF + 1
    o = rng.integers(0, reach, 200_000, dtype=np.uint64)
    for P, b in ((2, 20), (8, 20), (3, 7), (8, 16)):
        owner, local = D.block_owner_local(o, P, b)
        assert owner.min() >= 0 and owner.max() < P
        # bijective: (owner, local) -> o
        blk_local = local >> np.uint64(b)
        back = ((blk_local * np.uint64(P) + owner.astype(np.uint64)) << np.uint64(b)) | (local & np.uint64((1 << b) - 1))
        assert (back == o).all()
        for s in range(P):
            assert (local[owner == s] < np.uint64(D.shard_local_bits(reach, P, s, b))).all()
        # the probe-dense prefix [0, 2^32) is spread over every shard
        low = o[o < np.uint64(1 << 32)]
        lo_owner, _ = D.block_owner_local(low, P, b)
        assert len(set(lo_owner.tolist())) == P
    # interleave/split are inverse
    data = bytes(rng.integers(0, 256, 5000, dtype=np.uint8))
    data = data.rstrip(b"\0")
    parts = [D.split_shard(data, 3, s, 5000 * 8, 7) for s in range(3)]
    assert D.interleave_shards(parts, 5000 * 8, 7) == data


def test_sparse_checker_matches_dense_oracle():
    """The sparse comparison the 10B x 8 replicated GPU test uses (dist_worker.sparse_bits /
    sparse_include) equals the dense oracle's Redis string and include? answers."""
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import dist_worker as W
    import oracle as O
    orc = O.COracle()
    for m, k in ((95851, 6), (9585058, 6), (191701167547, 13)):
        keys = ["s%d" % i for i in range(700)]
        pos, val, idx = W.sparse_bits(orc, keys, m, k)
        probe = keys[::5] + ["n%d" % i for i in range(300)]
        got_inc = W.sparse_include(orc, idx, probe, m, k)
        if m < 10**8:
            bits = orc.new_bitset(m, k)
            kb, ko = O.pack_keys(keys)
            orc.insert_many(bits, m, k, kb, ko)
            s = np.frombuffer(orc.redis_string(bits), np.uint8)
            nz = np.flatnonzero(s)
            assert np.array_equal(nz, pos) and np.array_equal(s[nz], val)
            pb, po = O.pack_keys(probe)
            assert np.array_equal(orc.include_many(bits, m, k, pb, po).astype(bool), got_inc)
        assert got_inc[: len(keys[::5])].all()
