"""One rank of the multi-process partitioned-filter test (launched through
torch.distributed.run over gloo by tests/test_distributed.py on the CPU and by
tests/test_gpu_distributed.py on a GPU box).

The exchange logic under test is redis-bloomfilter_amd/distributed.py.  The
per-rank primitives come from a numpy engine built on the oracle (test
infrastructure) on the CPU, or — cfg "engine": "hip" — from libbfhip.so's
HipEngine with every rank on GPU 0 (gloo stages the device tensors through
host memory; RCCL refuses ranks that share a device).  Every rank checks the
assembled Redis string and every include? answer against a single-filter
oracle run over all ranks' keys.
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("BFHIP_STANDALONE", "1")

import pkgload  # noqa: E402
import oracle as O  # noqa: E402  (checker / reference engine only)

pkg = pkgload.load()
from redis_bloomfilter_amd import distributed as D  # noqa: E402
from ref_engine import NumpyEngine  # noqa: E402


def or_allreduce_case(rank, P, dev=None):
    """distributed.or_allreduce_ against the OR of every rank's tensor, for sizes that do
    not divide into P 16-byte chunks (dev: a device tensor, host-staged under gloo)."""
    ok = True
    for n in (1, 15, 1000, 4099):
        mine = torch.from_numpy(np.random.default_rng([n, rank]).integers(0, 256, n, dtype=np.uint8))
        t = mine.clone() if dev is None else mine.to(dev)
        D.or_allreduce_(t)
        t = t.cpu()
        want = np.zeros(n, np.uint8)
        for r in range(P):
            want |= np.random.default_rng([n, r]).integers(0, 256, n, dtype=np.uint8)
        ok = ok and bool((t.numpy() == want).all())
    return ok


def replicated_case(rank, P, cfg, dev):
    """ReplicatedFilter on the HIP engine: both insert forms (gather, OR-all-reduce) leave
    every replica's Redis string equal to one oracle filter over all ranks' keys, and the
    local include? answers equal the oracle's."""
    m, k = cfg["m"], cfg["k"]
    orc = O.COracle()
    keys = [["q%d-%d" % (r, int(v)) for v in np.random.default_rng([cfg["seed"], r]).integers(0, 10**9, cfg["n"])]
            for r in range(P)]
    all_keys = [x for ks in keys for x in ks]
    ib, io = O.pack_keys(all_keys)
    bits = orc.new_bitset(m, k)
    orc.insert_many(bits, m, k, ib, io)
    want_s = orc.redis_string(bits)
    probe = all_keys + ["fresh-%d-%d" % (rank, i) for i in range(cfg["n"])]
    pb, po = O.pack_keys(probe)
    want = orc.include_many(bits, m, k, pb, po).astype(bool)
    ok = True
    for mode in ("gather", "or", "digests", "sets"):
        rf = D.ReplicatedFilter(m, k, device=dev, insert_mode=mode)
        rf.insert_many(keys[rank])
        ok = ok and rf.last_insert_mode == mode and rf.export_redis() == want_s
        ok = ok and bool((rf.include_many(probe) == want).all())
        rf.close()
    # the pipelined form bench.py uses: the batch's gather started ahead of other work (here a
    # second gather in flight), then every rank's batch, this rank's included, as one insert
    half = len(keys[rank]) // 2
    kb1, ko1, n1 = D._device_batch(keys[rank][:half], dev)
    kb2, ko2, n2 = D._device_batch(keys[rank][half:], dev)
    for mode in ("gather", "or", "digests", "sets"):
        rf = D.ReplicatedFilter(m, k, device=dev, insert_mode=mode)
        st1 = rf.gather_start(kb1, ko1, n1)
        st2 = rf.gather_start(kb2, ko2, n2)
        rf.insert_gathered(st1)
        rf.insert_gathered(st2)
        ok = ok and rf.last_insert_mode == mode and rf.export_redis() == want_s
        rf.close()
    # uneven batches (rank r brings n - 50 r keys): every insert form pads and cuts correctly
    cut = [len(keys[r]) - 50 * r for r in range(P)]
    sub = [x for r in range(P) for x in keys[r][:cut[r]]]
    sb_, so_ = O.pack_keys(sub)
    ub = orc.new_bitset(m, k)
    orc.insert_many(ub, m, k, sb_, so_)
    want_u = orc.redis_string(ub)
    for mode in ("gather", "or", "digests", "sets"):
        rf = D.ReplicatedFilter(m, k, device=dev, insert_mode=mode)
        rf.insert_many(keys[rank][:cut[rank]])
        ok = ok and rf.export_redis() == want_u
        rf.close()
    # ... with the sizes all-gathered one batch ahead (sizes_start), as bench.py pipelines them
    rf = D.ReplicatedFilter(m, k, device=dev, insert_mode="gather")
    sz1 = rf.sizes_start(kb1, ko1, n1)
    sz2 = rf.sizes_start(kb2, ko2, n2)
    st1 = rf.gather_start(kb1, ko1, n1, sizes=sz1)
    rf.insert_gathered(st1)
    st2 = rf.gather_start(kb2, ko2, n2, sizes=sz2)
    rf.insert_gathered(st2)
    ok = ok and rf.export_redis() == want_s
    rf.close()
    return ok


class _DevBytes:
    """Raw device bytes (a filter's bitset) as a torch tensor, without a copy."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def sparse_bits(orc, keys, m, k):
    """The Redis string of inserting `keys` into an empty (m, k) filter, as (nonzero byte
    positions, their bytes), from the oracle's offsets alone: a 6.98 GB string need not be
    built to be compared, since an insert only ever sets bits (ruby.rb:57-60)."""
    kb, ko = O.pack_keys(keys)
    idx = np.unique(orc.indexes_many(kb, ko, m, k).reshape(-1))
    pos = (idx >> np.uint64(3)).astype(np.int64)
    mask = (np.uint64(0x80) >> (idx & np.uint64(7))).astype(np.uint8)
    starts = np.flatnonzero(np.concatenate([[True], pos[1:] != pos[:-1]]))
    return pos[starts], np.bitwise_or.reduceat(mask, starts), idx


def device_sparse(f):
    """(nonzero byte positions, bytes) of a filter's device bitset, found on the device."""
    torch.cuda.synchronize()
    ptr, nbytes = f.device_bits()
    t = torch.as_tensor(_DevBytes(ptr, nbytes), device="cuda")
    pos, val = [], []
    for a in range(0, nbytes, 1 << 28):   # torch.nonzero's scratch grows with its input: 256 MiB pieces
        nz = torch.nonzero(t[a: a + (1 << 28)]).view(-1) + a
        pos.append(nz.cpu().numpy())
        val.append(t[nz].cpu().numpy())
    return np.concatenate(pos), np.concatenate(val)


def sparse_include(orc, set_idx, probe, m, k):
    """The oracle's include? answers over a filter whose set bits are `set_idx` (sorted)."""
    pb, po = O.pack_keys(probe)
    idx = orc.indexes_many(pb, po, m, k).reshape(len(probe), k)
    return np.isin(idx, set_idx).all(axis=1)


def replicated_big_case(rank, P, cfg, dev):
    """BASELINE configs[3] (10B@0.01 %, 6.98 GB reachable, replicated on every rank, key
    batches sharded) through the forms bench.py --config 10b runs: the "digests" insert (each
    rank hashes its own batch once, the SHA-1 words are all-gathered, every replica inserts all
    of them from words as one binned insert), both through insert_many and through the
    pipelined sizes_start / gather_start(sizes=) / insert_gathered sequence, plus uneven
    batches; the "gather" form for comparison.  Every replica's bitset must equal the oracle's
    over all ranks' keys (compared sparsely, ruby.rb:57-63) and its include? answers the
    oracle's (ruby.rb:20-30)."""
    m, k, n = cfg["m"], cfg["k"], cfg["n"]
    orc = O.COracle()
    keys = [["q%d-%d" % (r, int(v)) for v in np.random.default_rng([cfg["seed"], r]).integers(0, 10**9, n)]
            for r in range(P)]
    all_keys = [x for ks in keys for x in ks]
    want_pos, want_val, set_idx = sparse_bits(orc, all_keys, m, k)
    probe = all_keys[rank::P] + ["fresh-%d-%d" % (rank, i) for i in range(n)]
    want_inc = sparse_include(orc, set_idx, probe, m, k)
    ok = True

    def same(rf, wp, wv):
        gp, gv = device_sparse(rf.filter)
        return bool(np.array_equal(gp, wp) and np.array_equal(gv, wv))

    for mode in ("digests", "sets", "gather"):
        rf = D.ReplicatedFilter(m, k, device=dev, insert_mode=mode)
        rf.insert_many(keys[rank])
        ok = ok and rf.last_insert_mode == mode and same(rf, want_pos, want_val)
        ok = ok and bool((rf.include_many(probe) == want_inc).all())
        rf.close()
        if not ok:
            print("rank %d replicated 10B mode %s MISMATCH" % (rank, mode), flush=True)
    # bench.py's pipelined step: batch i+1's sizes all-gathered one batch ahead, its words
    # gathered beside batch i's insert, then every rank's batch as one insert from words
    third = n // 3
    parts = [keys[rank][:third], keys[rank][third: 2 * third], keys[rank][2 * third:]]
    bt = [D._device_batch(p, dev) for p in parts]
    for mode in ("digests", "sets"):
        rf = D.ReplicatedFilter(m, k, device=dev, insert_mode=mode)
        szp = {0: rf.sizes_start(*bt[0]), 1: rf.sizes_start(*bt[1])}
        gpend = {0: rf.gather_start(*bt[0], sizes=szp.pop(0))}
        for i in range(3):
            st = gpend.pop(i)
            if i + 1 < 3:
                gpend[i + 1] = rf.gather_start(*bt[i + 1], sizes=szp.pop(i + 1))
            if i + 2 < 3:
                szp[i + 2] = rf.sizes_start(*bt[i + 2])
            rf.insert_gathered(st)
        ok = ok and rf.last_insert_mode == mode and same(rf, want_pos, want_val)
        ok = ok and bool((rf.include_many(probe) == want_inc).all())
        rf.close()
        if not ok:
            print("rank %d replicated 10B pipelined %s MISMATCH" % (rank, mode), flush=True)
    # uneven batches (rank r brings n - 50 r keys; the last rank none): the gathered words
    # are padded to the largest batch and the padding rows cut out before the insert
    cut = [n - 50 * r if r != P - 1 else 0 for r in range(P)]
    sub = [x for r in range(P) for x in keys[r][:cut[r]]]
    up, uv, _ = sparse_bits(orc, sub, m, k)
    for mode in ("digests", "sets"):
        rf = D.ReplicatedFilter(m, k, device=dev, insert_mode=mode)
        rf.insert_many(keys[rank][:cut[rank]])
        ok = ok and same(rf, up, uv)
        rf.close()
    if not ok:
        print("rank %d replicated 10B uneven MISMATCH" % rank, flush=True)
    # bench.py --gpus 8 --config 10b's own step (ReplicatedPipeline, fused hash, region sets)
    return rpipe_case(rank, P, dict(cfg, n=n // 2, steps=4), dev) and ok


def rpipe_case(rank, P, cfg, dev):
    """The exact replicated step bench.py --gpus N times on the replicated layouts
    (distributed.ReplicatedPipeline): step i's include? kernel hashes batch
    i+2 into a ring of three word buffers, step i+1 encodes those words into region sets
    (gather_start(..., digests=)) and all-gathers them while batch i+2's sizes travel, step i+2
    ORs every rank's sets in (insert_gathered, "sets"), and the last step's gather wraps around
    to batch 0.  After every step the include? answers must equal the oracle's over every
    rank's batches 0..i (ruby.rb:20-30); after the last, every replica's bitset must equal the
    oracle's over all of them (ruby.rb:57-63), compared sparsely.  Then: a damaged set buffer
    makes every rank raise at its sets check, and a batch one encode cannot take
    on one rank moves every rank to the digests form for that batch."""
    m, k, n, L = cfg["m"], cfg["k"], cfg["n"], cfg.get("steps", 5)
    orc = O.COracle()

    def ins_keys(r, b):
        return ["p%d-%d-%d" % (r, b, int(v)) for v in np.random.default_rng([cfg["seed"], r, b]).integers(0, 10**12, n)]

    def inc_keys(r, b):   # half that step's inserts, half fresh
        return ins_keys(r, b)[: n // 2] + ["np%d-%d-%d" % (r, b, i) for i in range(n - n // 2)]

    batches = [(D._device_batch(ins_keys(rank, b), dev)[:2], D._device_batch(inc_keys(rank, b), dev)[:2])
               for b in range(L)]
    rf = D.ReplicatedFilter(m, k, device=dev, insert_mode="sets")
    rpl = D.ReplicatedPipeline(rf, batches, n, fused_hash=True)
    outs = []
    for _ in range(L):
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        rpl.insert()
        rpl.include(out)
        outs.append(out)
    torch.cuda.synchronize()
    rpl.drain()
    ok = rf.last_insert_mode == "sets"
    rf.sets_check()
    set_idx = np.zeros(0, np.uint64)
    for b in range(L):   # the answers of step b see every rank's batches 0..b
        keys_b = [x for r in range(P) for x in ins_keys(r, b)]
        kb_, ko_ = O.pack_keys(keys_b)
        set_idx = np.union1d(set_idx, orc.indexes_many(kb_, ko_, m, k).reshape(-1))
        want = sparse_include(orc, set_idx, inc_keys(rank, b), m, k)
        good = bool((outs[b].cpu().numpy().astype(bool) == want).all())
        if not good:
            print("rank %d rpipe step %d: %d answers differ" % (rank, b, int((outs[b].cpu().numpy().astype(bool) != want).sum())),
                  flush=True)
        ok = ok and good
    all_keys = [x for b in range(L) for r in range(P) for x in ins_keys(r, b)]
    want_pos, want_val, _ = sparse_bits(orc, all_keys, m, k)
    gp, gv = device_sparse(rf.filter)
    same = bool(np.array_equal(gp, want_pos) and np.array_equal(gv, want_val))
    if not same:
        print("rank %d rpipe: bitset differs from the oracle" % rank, flush=True)
    ok = ok and same
    rf.close()
    # a damaged buffer (the last rank's header) is skipped by every replica, and every rank
    # raises at its next sets check instead of answering false for inserted keys later
    rf = D.ReplicatedFilter(m, k, device=dev, insert_mode="sets")
    st = rf.gather_start(*batches[0][0], n)
    for w in st["works"]:
        w.wait()
    st["gs"].view(P, -1)[P - 1, 0] = 0
    rf.insert_gathered(st)
    try:
        rf.sets_check()
        ok = False
        print("rank %d: a damaged set buffer went unreported" % rank, flush=True)
    except pkg.BfHipError:
        pass
    rf.close()
    # rank 0's batch past what one encode takes (here: a capacity bound lowered to below it):
    # every rank learns it from the gathered sizes and takes the digests form for that batch
    rf = D.ReplicatedFilter(m, k, device=dev, insert_mode="sets")
    real = rf.filter.region_sets_capacity
    lim = n // 2

    def capped(nk):
        if nk > lim:
            raise pkg.ArgumentError("test: %d keys past one encode" % nk)
        return real(nk)

    rf.filter.region_sets_capacity = capped
    mine = ins_keys(rank, 0)[: (n if rank == 0 else lim)]
    rf.insert_many(mine)
    ok = ok and rf.last_insert_mode == "digests"
    rf.insert_many(ins_keys(rank, 1)[:lim])
    ok = ok and rf.last_insert_mode == "sets"
    sub = [x for r in range(P) for x in ins_keys(r, 0)[: (n if r == 0 else lim)]]
    sub += [x for r in range(P) for x in ins_keys(r, 1)[:lim]]
    up, uv, _ = sparse_bits(orc, sub, m, k)
    gp, gv = device_sparse(rf.filter)
    fb = bool(np.array_equal(gp, up) and np.array_equal(gv, uv))
    if not fb:
        print("rank %d: the digests fallback differs from the oracle" % rank, flush=True)
    rf.close()
    return ok and fb


def uneven_case(rank, P, cfg, dev, make_engine):
    """Ranks that bring batches of different sizes (the sync-free windows must
    not be sized from a rank's own n), one rank bringing none, and a later batch past the
    agreed bound on one rank only (its windows overflow, every rank replays through the
    synced path and the bound rises).  Shard bytes and answers must equal the oracle's."""
    m, k = cfg["m"], cfg["k"]
    orc = O.COracle()
    sizes = [cfg["n"] + 97 * r if r != P - 1 or P < 3 else 0 for r in range(P)]

    def keys_of(r, n, tag):
        return ["%s%d-%d" % (tag, r, int(v)) for v in np.random.default_rng([cfg["seed"], r, n]).integers(0, 10**9, n)]

    pf = D.PartitionedFilter(m, k, block_log2=cfg["block_log2"], engine=make_engine())
    pf.insert_many(keys_of(rank, sizes[rank], "a"))                      # agrees on max n
    probe1 = keys_of(rank, sizes[rank], "a")[: sizes[rank] // 2] + keys_of(rank, 50 + 13 * rank, "x")
    got1 = pf.include_many(probe1)
    # the bench's cross-step form with uneven batches (next_insert prefetched)
    kb1, ko1, n1 = D._device_batch(keys_of(rank, sizes[rank] // 3, "b"), dev or "cpu")
    kb2, ko2, n2 = D._device_batch(keys_of(rank, 7 * rank + 5, "c"), dev or "cpu")
    probe2 = keys_of(rank, 40 + rank, "b") + keys_of(rank, sizes[rank] // 3, "b")[:20]
    qkb, qko, nq = D._device_batch(probe2, dev or "cpu")
    pf.insert_include_dev(kb1, ko1, n1, qkb, qko, nq, next_insert=(kb2, ko2, n2))
    got2 = pf.insert_include_dev(kb2, ko2, n2, qkb, qko, nq).cpu().numpy().astype(bool)
    agreed = pf._sf_n
    # rank 0 twice past its windows at the agreed bound (every window holds ~1/(P nh) of the probes)
    nwin = P * getattr(pf.engine, "nh", 1)
    big = [2 * pf._cap_sf(agreed) * nwin // k + 1 if r == 0 else cfg["n"] // 2 for r in range(P)]
    # rank 0 alone past the bound: a global overflow, a synced replay, a raised bound
    pf.insert_many(keys_of(rank, big[rank], "d"))
    probe3 = keys_of(rank, big[rank], "d")[::3] + keys_of(rank, 30, "y")
    got3 = pf.include_many(probe3)
    ok = pf.replays >= 1 and pf._sf_n >= max(big) and agreed == max(sizes)
    # the oracle over every rank's keys
    allk = []
    for r in range(P):
        allk += keys_of(r, sizes[r], "a") + keys_of(r, sizes[r] // 3, "b") + keys_of(r, 7 * r + 5, "c")
        allk += keys_of(r, big[r], "d")
    ib, io = O.pack_keys(allk)
    bits = orc.new_bitset(m, k)
    orc.insert_many(bits, m, k, ib, io)
    want_s = orc.redis_string(bits)
    s = pf.export_redis()
    ok = ok and ((s == want_s) if rank == 0 else s is None)
    # answers: probe1 after the "a" inserts only, probe2 after a+b+c... — recompute in order
    def answers(ins_sets, probe):
        b2 = orc.new_bitset(m, k)
        ks = [x for r in range(P) for fn in ins_sets for x in fn(r)]
        kb_, ko_ = O.pack_keys(ks)
        orc.insert_many(b2, m, k, kb_, ko_)
        pb, po = O.pack_keys(probe)
        return orc.include_many(b2, m, k, pb, po).astype(bool)
    a_ = lambda r: keys_of(r, sizes[r], "a")
    b_ = lambda r: keys_of(r, sizes[r] // 3, "b")
    c_ = lambda r: keys_of(r, 7 * r + 5, "c")
    d_ = lambda r: keys_of(r, big[r], "d")
    ok = ok and bool((got1 == answers([a_], probe1)).all())
    ok = ok and bool((got2 == answers([a_, b_, c_], probe2)).all())
    ok = ok and bool((got3 == answers([a_, b_, c_, d_], probe3)).all())
    if not ok:
        print("rank %d uneven MISMATCH: replays %d agreed %s bound %s" % (rank, pf.replays, agreed, pf._sf_n),
              flush=True)
    # a pending prefetch blocks the whole-filter calls; a mismatched consume is refused and
    # leaves the prefetch pending (no rank runs a collective alone) until every rank drains it
    pf.insert_include_dev(kb1, ko1, n1, qkb, qko, nq, next_insert=(kb2, ko2, n2))
    try:
        pf.clear()
        ok = False
    except pkg.ArgumentError:
        pass
    try:
        pf.insert_include_dev(kb1, ko1, n1, qkb, qko, nq)
        ok = False
    except pkg.ArgumentError:
        pass
    ok = ok and pf._pending is not None
    pf.drain_prefetch()
    ok = ok and pf._pending is None
    pf.clear()
    pf.close()
    return ok


def main():
    dist.init_process_group("gloo")
    rank, P = dist.get_rank(), dist.get_world_size()
    cfg = json.loads(os.environ["BF_DIST_CFG"])
    hip = cfg.get("engine") == "hip"
    dev = torch.device("cuda", 0) if hip else None
    if cfg.get("case") in ("replicated", "replicated_big", "rpipe"):
        fn = {"replicated": replicated_case, "replicated_big": replicated_big_case, "rpipe": rpipe_case}[cfg["case"]]
        flag = torch.tensor([1 if fn(rank, P, cfg, dev) else 0])
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if rank == 0:
            print("DIST_RESULT", "ok" if flag.item() == 1 else "fail", flush=True)
        dist.destroy_process_group()
        sys.exit(0 if flag.item() == 1 else 1)
    if cfg.get("case") == "or_allreduce":
        flag = torch.tensor([1 if or_allreduce_case(rank, P, dev) else 0])
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if rank == 0:
            print("DIST_RESULT", "ok" if flag.item() == 1 else "fail", flush=True)
        dist.destroy_process_group()
        sys.exit(0 if flag.item() == 1 else 1)
    m, k, b = cfg["m"], cfg["k"], cfg["block_log2"]

    def engine(m, k, P, rank, b, orc, dev):
        return D.HipEngine(m, k, P, rank, b, dev) if dev is not None else NumpyEngine(m, k, P, rank, b, orc)

    orc = O.COracle()
    if cfg.get("case") == "uneven":
        flag = torch.tensor([1 if uneven_case(rank, P, cfg, dev, lambda: engine(m, k, P, rank, b, orc, dev)) else 0])
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if rank == 0:
            print("DIST_RESULT", "ok" if flag.item() == 1 else "fail", flush=True)
        dist.destroy_process_group()
        sys.exit(0 if flag.item() == 1 else 1)
    pf = D.PartitionedFilter(m, k, block_log2=b, engine=engine(m, k, P, rank, b, orc, dev))
    assert pf.sync_free
    rng = np.random.default_rng([cfg["seed"], rank])
    mine = [("r%d-%d" % (rank, int(v))) for v in rng.integers(0, 10**9, cfg["n"])]
    pf.insert_many(mine)
    probe = ["r%d-%d" % (r, int(v)) for r in range(P)
             for v in np.random.default_rng([cfg["seed"], r]).integers(0, 10**9, cfg["n"])]
    probe += ["fresh-%d-%d" % (rank, i) for i in range(cfg["n"])]
    got = pf.include_many(probe)
    # the single-filter oracle over every rank's keys (each rank computes it)
    all_keys = [("r%d-%d" % (r, int(v))) for r in range(P)
                for v in np.random.default_rng([cfg["seed"], r]).integers(0, 10**9, cfg["n"])]
    ib, io = O.pack_keys(all_keys)
    bits = orc.new_bitset(m, k)
    orc.insert_many(bits, m, k, ib, io)
    want_s = orc.redis_string(bits)
    del bits
    s = pf.export_redis()                    # assembled on rank 0 only
    export_ok = (s == want_s) if rank == 0 else (s is None)
    write_ok = True
    if pf.reach_bits <= (1 << 31):
        # per-rank SETRANGE of each rank's own blocks into "Redis" (here one FakeRedis per
        # process, merged below by OR, since each rank only writes its own blocks)
        r = pkg.FakeRedis(max_string=1 << 40)
        if rank == 0:
            r.set("bf", b"stale")            # replace: rank 0 DELs first (the shared key)
        pf.write_redis(r, "bf", chunk_bytes=4096)
        parts = [None] * P
        dist.all_gather_object(parts, r.get("bf") or b"")
        width = max(len(x) for x in parts)
        merged = np.zeros(width, np.uint8)
        for x in parts:
            merged[: len(x)] |= np.frombuffer(x, np.uint8)
        write_ok = merged.tobytes() == want_s and width == len(want_s)
    s = want_s if rank != 0 else s
    # round trip: a fresh partitioned filter loaded from the string answers identically
    pf2 = D.PartitionedFilter(m, k, block_log2=b, engine=engine(m, k, P, rank, b, orc, dev))
    pf2.import_redis(s)
    got2 = pf2.include_many(probe)
    # the overlapped insert + include? step gives the sequential form's shard bytes and answers
    del pf2   # the 10B case holds 3.5 GB per shard copy
    pf3 = D.PartitionedFilter(m, k, block_log2=b, engine=engine(m, k, P, rank, b, orc, dev))
    got3 = pf3.insert_include(mine, probe)
    same_shard = bool(np.array_equal(pf3.engine.shard_export(), pf.engine.shard_export()))
    # the first overlapped call agrees on its bound from both batches (the include? batch is
    # the larger here), so nothing overflows; cfg "chunks": whether this shard count takes
    # chunked windows (P * nh past the directory limit falls back to plain windows)
    same_shard = same_shard and pf3.replays == 0 and pf3.chunks == cfg.get("chunks", pf3.chunks)
    if not same_shard:
        print("rank %d pf3: replays %d chunks %s" % (rank, pf3.replays, pf3.chunks), flush=True)
    shard_sha = hashlib.sha1(pf.engine.shard_export().tobytes()).hexdigest()
    del pf, pf3
    # the same step through the contiguous route (windows off), and with every window
    # overflowing (each rank falls back to the contiguous route after the count exchange)
    # ... and through the synced exchange (host waits for the counts), the sync-free one with
    # every window overflowing (the batch is replayed through the synced path), and bytes
    # instead of bits on the way back
    got45 = []
    for kw, cap in (({"windows": False}, None), ({"sync_free": False}, 3), ({}, "sf"),
                    ({"pack_answers": False}, None), ({"pack_answers": False, "sync_free": False}, None)):
        pf4 = D.PartitionedFilter(m, k, block_log2=b, engine=engine(m, k, P, rank, b, orc, dev), **kw)
        if cap == "sf":
            pf4._cap_sf = lambda n: 8
        elif cap is not None:
            pf4._cap = lambda n, c=cap: c
        got45.append(pf4.insert_include(mine, probe))
        same_shard = same_shard and hashlib.sha1(pf4.engine.shard_export().tobytes()).hexdigest() == shard_sha
        if cap == "sf":
            same_shard = same_shard and pf4.sync_free and pf4.replays == 1
        elif cap is not None:
            same_shard = same_shard and pf4.window_overflows == 2
        del pf4
    # the cross-step form bench.py uses: the next call's insert batch routed and sent during
    # this call (next_insert), then consumed by the next call; a prefetch no call consumes
    # is completed by drain_prefetch
    half = len(mine) // 2
    kb1, ko1, n1 = D._device_batch(mine[:half], dev or "cpu")
    kb2, ko2, n2 = D._device_batch(mine[half:], dev or "cpu")
    qkb, qko, nq = D._device_batch(probe, dev or "cpu")
    pf6 = D.PartitionedFilter(m, k, block_log2=b, engine=engine(m, k, P, rank, b, orc, dev))
    # (next_include: the first call's owner test hashes the second call's include? batch, which
    # the second call then routes from the words — the chunked HIP engine's P = 8 form)
    pf6.insert_include_dev(kb1, ko1, n1, qkb, qko, nq, next_insert=(kb2, ko2, n2), next_include=(qkb, qko, nq))
    words_ready = pf6._next_inc is not None or not pf6.chunks
    got6 = pf6.insert_include_dev(kb2, ko2, n2, qkb, qko, nq, next_insert=(kb1, ko1, n1))
    # ... and the second call's include? route really started from those words
    routed_from_words = words_ready and (not pf6.chunks or pf6.routed_from_digests == 1)
    same_shard = same_shard and routed_from_words
    pf6.drain_prefetch()
    got6 = got6.cpu().numpy().astype(bool)
    same_shard = same_shard and hashlib.sha1(pf6.engine.shard_export().tobytes()).hexdigest() == shard_sha
    del pf6
    got45.append(got6)
    ok = True
    if rank == 0 or True:
        bits = orc.new_bitset(m, k)
        orc.insert_many(bits, m, k, ib, io)
        pb, po = O.pack_keys(probe)
        want = orc.include_many(bits, m, k, pb, po).astype(bool)
        ok = export_ok and same_shard and write_ok and bool((got == want).all()) \
            and bool((got2 == want).all()) and bool((got3 == want).all()) and all(bool((g == want).all()) for g in got45)
        if not ok:
            print("rank %d MISMATCH: export %s, write_redis %s, include %d diffs" %
                  (rank, export_ok, write_ok, int((got != want).sum())), flush=True)
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        print("DIST_RESULT", "ok" if flag.item() == 1 else "fail", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if flag.item() == 1 else 1)


if __name__ == "__main__":
    main()
