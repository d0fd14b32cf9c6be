#!/usr/bin/env python3
"""Throughput bench for the Bloom-filter hot path (insert_many + include_many?).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config nstar|1m|100m|10k]

One step = one ``insert_many`` batch + one ``include_many?`` batch of B
synthetic keys each (key family D: decimal strings of seeded uniform ints,
bf_100_000_flat.rb:21-22), inputs already resident in HBM, launched through
the C ABI's device entry points on torch's current stream.  The include?
batch is 50 % keys of the insert batch and 50 % fresh keys.

Default workload (``nstar``): the north-star filter of BASELINE.json — 1B keys
at 1 % error, m = 9,585,058,377 bits (1.20 GB), k = 6 — prefilled to 50 % bit
density, B = 2^24 keys per batch.  It is the configuration the metric's
"% of HBM random-access roofline" is quoted on; the cache-resident configs
(1M@1 %, 100M@0.1 %) are reported under ``secondary``.

Multi-GPU (``--gpus N`` under torch.distributed.run): the filter is
block-partitioned over the N GPUs and every rank brings its own key batches
(weak scaling); probes travel to their owner GPU by RCCL all-to-all and
include? answers come back the same way (redis-bloomfilter_amd/distributed.py).

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402   (imported before libbfhip: one shared HIP runtime)
import torch.distributed as dist  # noqa: E402

import pkgload  # noqa: E402

HBM_PEAK = 8.0e12          # B/s, MI355X_MICROARCH.md chip table (spec)
GRANULE = 64               # B per random probe (SURVEY §8 d)
# Random 4-B probes of a buffer past L2 leave it as 128-B line fills whatever the memory type
# or cache policy, at ~55 G fills/s for any working set from 64 MiB to 1.2 GB (Infinity Cache
# residency does not raise it): tools/probe_granularity.hip, profiles/r02_probe_granularity.log
FILL_CEILING = 55.1e9      # fills/s, plain loads, 1143 MiB working set
# ... and 50.2 G/s over 6656 MiB, the reach-capped 10B / 200B bitsets (profiles/r02z_probe_sweep.log)
FILL_CEILING_7GB = 50.2e9


# ... and 258 G/s over a 2 MiB working set (L2-resident: the Lua layout's 1.38 MB first layer at
# 1M@1 %, profiles/r02z_probe_sweep.log line 1)
FILL_CEILING_L2 = 258.4e9


def fill_ceiling(bitset_bytes: int):
    """The measured random-fill ceiling for a bitset of this size, and its source."""
    if bitset_bytes > (2 << 30):
        return FILL_CEILING_7GB, "tools/probe_granularity.hip sweep, 6656 MiB (profiles/r02z_probe_sweep.log)"
    return FILL_CEILING, "tools/probe_granularity.hip (profiles/r02_probe_granularity.log)"
SEED = 0x5EED

CONFIGS = {
    # name: (n, error_rate, batch, prefill)
    "nstar": (10**9, 0.01, 1 << 24, "random"),
    "100m": (10**8, 0.001, 1 << 24, "random"),
    "1m": (10**6, 0.01, 1 << 20, "insert"),
    "10k": (10**4, 0.01, 1 << 14, "insert"),
    # hash-bound probe: the 1M@1% (L2-resident) filter driven with 2^24-key batches
    "1m_big": (10**6, 0.01, 1 << 24, "insert"),
    # BASELINE configs 4 and 5 on one GPU: their reachable prefix (k(2^32-1)+1 bits, 6.98 GB,
    # ruby.rb:51) fits one MI355X; the 8-GPU layouts are --gpus 8 runs
    "10b": (10**10, 0.0001, 1 << 24, "random"),
    "200b": (2 * 10**11, 0.0001, 1 << 24, "random"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Dist:
    """One process per GPU.  backend "nccl" (RCCL over xGMI) is the measured path; "gloo"
    is a rehearsal of the same multi-rank step with host-staged exchanges (distributed.py),
    which also runs several ranks on one GPU (rank r on device r % device_count) — what a
    one-GPU box can check of the N > 1 path; its times say nothing about xGMI."""

    def __init__(self, need_group: bool = False, backend: str = "nccl", no_device: bool = False):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = backend
        if no_device:   # --launch-check: the process group alone (gloo), no GPU touched
            self.group = self.world > 1 or need_group
            if self.group:
                dist.init_process_group(backend="gloo")
            return
        if backend == "gloo":
            self.local %= max(torch.cuda.device_count(), 1)
        self.group = self.world > 1 or need_group
        if self.group:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if self.world == 1:
                import socket
                sk = socket.socket()
                sk.bind(("127.0.0.1", 0))
                os.environ.setdefault("MASTER_PORT", str(sk.getsockname()[1]))
                sk.close()
                os.environ.setdefault("RANK", "0")
                os.environ.setdefault("WORLD_SIZE", "1")
            torch.cuda.set_device(self.local)
            if backend == "nccl":
                dist.init_process_group(backend="nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group(backend=backend)
        else:
            torch.cuda.set_device(0)

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda" if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.group:
            dist.destroy_process_group()


_POW10 = {}


def pack_decimal_dev(vals: torch.Tensor):
    """``Integer#to_s`` + pack on the device (bench input synthesis, outside the timed region).

    vals: non-negative int64 on the GPU -> (uint8 key bytes + 16 B slack, int64 offsets[n+1])."""
    dev = vals.device
    if dev not in _POW10:
        _POW10[dev] = torch.tensor([10 ** i for i in range(19)], dtype=torch.int64, device=dev)
    pow10 = _POW10[dev]
    ndig = torch.searchsorted(pow10, vals, right=True).clamp_(min=1)
    width = int(ndig.max().item())
    div = pow10[:width].flip(0)
    digits = (torch.div(vals[:, None], div[None, :], rounding_mode="floor") % 10 + 48).to(torch.uint8)
    keep = torch.arange(width, device=dev)[None, :] >= (width - ndig)[:, None]
    buf = digits[keep]
    offs = torch.zeros(vals.numel() + 1, dtype=torch.int64, device=dev)
    torch.cumsum(ndig, 0, out=offs[1:])
    kb = torch.cat([buf, torch.zeros(16, dtype=torch.uint8, device=dev)])
    return kb, offs


def make_batches(n_filter: int, batch: int, rank: int, count: int, dev):
    """`count` step batches, each a fresh insert batch (uniform ints in [0, n)) and an
    include? batch of half that step's inserts + half fresh non-members (ints in [n, 2n))."""
    g = torch.Generator(device=dev)
    g.manual_seed(SEED * 1000 + rank)
    out = []
    for _ in range(count):
        ins = torch.randint(0, n_filter, (batch,), generator=g, device=dev, dtype=torch.int64)
        fresh = torch.randint(n_filter, 2 * n_filter, (batch - batch // 2,), generator=g, device=dev,
                              dtype=torch.int64)
        inc = torch.cat([ins[: batch // 2], fresh])
        out.append((pack_decimal_dev(ins), pack_decimal_dev(inc)))
    return out


def lua_config(pkg, D: Dist, reps: int = 5, entries: int = 10**6, precision: float = 0.01, batch: int = 1 << 20):
    """SURVEY §8 f1 on the device at the README's 1M scale (README.md:84-87 quotes the lua driver
    at 1M items): the scalable layout of lua.rb / add.lua / check.lua for entries = 1M,
    precision = 1 % (layer 1: 11,028,238 bits = 1.38 MB, k = 7), device-resident keys.  One rep
    = a fresh filter, bf_lua_insert_many_dev of 2^20 keys (decimal strings of uniform ints in
    [0, 1M): the bf_100_000_flat.rb shape at 1M) with add.lua's sequential semantics, then
    bf_lua_include_many_dev of 2^20 keys (half that batch, half fresh).  The insert returns once
    the count is known (the layer choice needs it); the timing brackets both calls with a device
    sync.  Median of `reps` reps after one warm-up rep; kernel times per layer by bf_lua_profile."""
    dev = torch.device("cuda", D.local)
    batches = make_batches(entries, batch, D.rank, reps + 1, dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    out = torch.empty(batch, dtype=torch.uint8, device=dev)
    flags = torch.empty(batch, dtype=torch.uint8, device=dev)
    f = pkg.LuaFilter(entries, precision, device=D.local)
    t_ins, t_inc, counts, layers = [], [], [], []
    for i, ((ikb, iko), (pkb, pko)) in enumerate(batches):
        f.clear()
        if i == 1:
            f.profile(True)
            f.profile_read(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), batch, flags.data_ptr(), stream=st)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        f.include_many_dev(pkb.data_ptr(), pko.data_ptr(), batch, out.data_ptr(), stream=st)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        assert bool(out[: batch // 2].all().item()), "lua_1m: an inserted key answered false"
        if i:
            t_ins.append(t1 - t0)
            t_inc.append(t2 - t1)
            counts.append(f.count)
            layers.append(f.layers)
    prof = f.profile_read(reset=True)
    f.profile(False)
    fp = float(out[batch // 2:].float().mean().item())
    f.close()
    ti, tc = sorted(t_ins)[len(t_ins) // 2], sorted(t_inc)[len(t_inc) // 2]
    bits1, k1 = pkg._lib.lua_layer_params(entries, precision, 1)
    # check.lua's probes (layer 1 only while count <= entries): members all k, non-members up to
    # their first 0 bit (density d = fp^(1/k) from the batch's observed false-positive rate)
    d = fp ** (1.0 / k1) if fp > 0 else 0.0
    per_key = 0.5 * k1 + 0.5 * ((1 - fp) / (1 - d) if d < 1 else k1)
    kern = {nm: {"ms": tot / cnt, "launches": cnt} for nm, (tot, cnt) in prof.items()}
    chk = kern.get("lua_check")
    return {"keys_per_s": 2 * batch / (ti + tc), "insert_keys_per_s": batch / ti, "include_keys_per_s": batch / tc,
            "insert_ms": ti * 1e3, "include_ms": tc * 1e3, "batch": batch, "entries": entries,
            "precision": precision, "count_after_insert": int(np.median(counts)), "layers": int(max(layers)),
            "layer1_bits": bits1, "layer1_k": k1, "layer1_bytes": (bits1 + 7) // 8,
            "kernels": {nm: round(v["ms"], 4) for nm, v in kern.items()},
            "include_fills": {"fills_per_key": per_key, "observed_fp_rate": fp,
                              "fills_per_s": batch * per_key / (chk["ms"] / 1e3) if chk else None,
                              "ceiling_fills_per_s": FILL_CEILING_L2,
                              "frac": batch * per_key / (chk["ms"] / 1e3) / FILL_CEILING_L2 if chk else None,
                              "ceiling_source": "tools/probe_granularity.hip sweep, 2 MiB working set "
                                                "(profiles/r02z_probe_sweep.log): the 1.38 MB layer is "
                                                "L2-resident, so SHA-1 (VALU), not fills, bounds it"},
            "timing": "median of %d reps, each on a fresh filter, wall time of each device call incl. its "
                      "syncs (the insert reads the count back per chunk)" % len(t_ins),
            "pmc": load_pmc("lua_1m")}


def to_host(kb: torch.Tensor, ko: torch.Tensor):
    offs = ko.cpu().numpy().view(np.uint64)
    return kb.cpu().numpy()[: int(offs[-1])], offs


class _DevBytes:
    """A torch view of raw device bytes (the filter's bitset) via __cuda_array_interface__."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def prefill_random(f, m: int, k: int, rank: int, host_copy: bool = True):
    """50 % bit density over the reachable prefix (a full filter holds 1 - e^{-kn/m} ~ 46.5 %).
    host_copy=False fills on the device (multi-GB secondary configs) and returns None."""
    nbytes = (f.reach_bits + 7) // 8
    if not host_copy:
        ptr, _ = f.device_bits()
        t = torch.as_tensor(_DevBytes(ptr, nbytes), device="cuda")
        g = torch.Generator(device=t.device)
        g.manual_seed(SEED * 7919 + rank)
        t.random_(0, 256, generator=g)
        tail = f.reach_bits & 7
        if tail:
            t[-1:].bitwise_and_((0xFF << (8 - tail)) & 0xFF)
        torch.cuda.synchronize()
        return None
    rng = np.random.default_rng([SEED, 99, rank])
    host = np.frombuffer(rng.bytes(nbytes), dtype=np.uint8).copy()
    tail = f.reach_bits & 7
    if tail:
        host[-1] &= (0xFF << (8 - tail)) & 0xFF
    f.import_redis(host.tobytes() if nbytes < (1 << 20) else memoryview(host))
    return host


# The replicated layout's insert form per config (ReplicatedFilter insert_mode; "auto" picks
# key bytes or the OR-all-reduce by size).  10B@0.01 % (BASELINE configs[3], k = 13): region
# sets — each rank sorts and encodes its own batch once, every replica ORs all ranks' sets in
# one pass: one replica's step 17.8 -> 12.5 ms against the SHA-1 words form on the same box
# (tools/sim_rank.py --replicated 8: profiles/r04b_sim_replicated.jsonl).  The north-star
# filter at N = 2 (the driver's N = 2 layout) too: 3.35 ms per replica step against 3.54 for the
# key gather, and 122 MB on the wire per rank against ~168 MB of key bytes
# (profiles/r04k_sim_replicated.jsonl, r04e_sim_replicated.jsonl).
REPLICATED_INSERT = {"10b": "sets", "nstar": "sets"}


def auto_mode(world: int, m: int, k: int, config: str = "nstar") -> str:
    """single at N = 1.  BASELINE's own layouts for its multi-GPU configs: 10b (configs[3],
    "10B keys replicated on 8 GPUs, key batches sharded") replicated, 200b (configs[4])
    partitioned.  Otherwise replicated at N = 2 for a filter that fits one GPU, where one
    xGMI link carries the whole exchange: the replicated step moves ~10 B per key once (key
    bytes + a length byte) against ~24 B per key out and back for the partitioned one, and
    its extra compute (each replica hashes both batches) is what the partitioned owner-side
    sort costs anyway; partitioned from N = 4 on, where the replicas' N-fold insert work
    loses (a replicated 1.2 GB filter cannot take the OR-reduce form either: 2.4 GB of
    bitset on the wire per step against ~1.3 GB of gathered keys)."""
    if world == 1:
        return "single"
    if config == "10b":
        return "replicated"
    if config == "200b":
        return "partitioned"
    reach_bytes = (min(m, k * 0xFFFFFFFF + 1) + 7) // 8
    return "replicated" if world == 2 and reach_bytes <= (64 << 30) else "partitioned"


def time_config(pkg, D: Dist, name: str, steps: int, warmup: int, want_host=False, mode: str = "auto",
                overlap: bool = True, pipeline: bool = False, comm_prefetch: bool = False,
                replicated_insert: str = "auto"):
    n, p, batch, prefill = CONFIGS[name]
    B = pkg.Bloomfilter
    m = B.optimal_m(n, p)
    k = B.optimal_k(n, m)
    dev = torch.device("cuda", D.local)
    t0 = time.time()
    pf = None
    host_bits = None
    if mode == "auto":
        mode = auto_mode(D.world, m, k, name)
    rf = None
    if mode == "replicated":   # every rank a whole replica: include? local, inserts all-gathered
        if replicated_insert == "auto":
            replicated_insert = REPLICATED_INSERT.get(name, "auto")
        rf = pkg.distributed.ReplicatedFilter(m, k, device=dev, insert_mode=replicated_insert)
        f = rf.filter
        if prefill == "random":   # identical replicas: the same bits on every rank
            prefill_random(f, m, k, 0, host_copy=f.device_bytes < (4 << 30))
    elif mode == "single":
        f = pkg.Filter(m, k, device=D.local)
        if prefill == "random":
            host_bits = prefill_random(f, m, k, D.rank, host_copy=f.device_bytes < (4 << 30))
    else:   # partitioned over the ranks, RCCL all-to-all routing
        pf = pkg.distributed.PartitionedFilter(m, k, block_log2=20, device=dev)
        f = pf.engine.filter
        if prefill == "random":
            rng = np.random.default_rng([SEED, 99, D.rank])
            f.shard_import(rng.bytes(f.local_bits // 8))
    batches = make_batches(n, batch, D.rank, warmup + steps, dev)
    torch.cuda.synchronize()
    log("[%s] m=%d k=%d batch=%d setup %.1fs" % (name, m, k, batch, time.time() - t0))
    out = torch.empty(batch, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream   # 0 = the null stream torch uses by default
    # replicated "sets" insert, pipelined: batch i+2's SHA-1 words come out of step i's include?
    # kernel (bf_include_hash_dev, as the single-GPU step), step i+1 encodes them into region sets
    # (no hash pass) and all-gathers them beside its own work, step i+2 ORs every rank's sets in
    rpipe = pipeline and rf is not None and comm_prefetch and rf.insert_mode == "sets"
    pipeline = pipeline and mode == "single"
    if pipeline:
        # Pipelined steps (include/bfhip.h, bf_include_hash_dev): step i inserts batch i from
        # its SHA-1 words (bf_insert_digests_dev: no hash pass), then answers include? batch i
        # while hashing insert batch i+1 in the same kernel — the include? waits on its probes'
        # memory latency and the hashing fills its idle VALUs.  Same work per step (one hash of
        # each key, one insert of 2^24 keys, one include? of 2^24 keys after it) and the same
        # answers (tests/test_gpu_digests.py::test_pipelined_steps_equal_plain_steps); the
        # last step hashes batch 0's keys again so that every step does the same work.
        digs = [torch.empty((batch, 4), dtype=torch.int32, device=dev) for _ in range(2)]
        ikb0, iko0 = batches[0][0]
        f.hash_many_dev(ikb0.data_ptr(), iko0.data_ptr(), batch, digs[0].data_ptr(), stream=sp)
        step_no = [0]

    # Replicated, comm_prefetch (distributed.ReplicatedPipeline, the code the multi-rank oracle
    # test runs: tests/dist_worker.py rpipe_case): step i starts the all-gather of batch i+1
    # before its own work, so the exchange runs beside step i's inserts and include? (the
    # process group's stream); step i then inserts every rank's batch i — its own with the
    # others, as ONE insert — before its include?, so every answer still sees all of the step's
    # inserts.  The last step gathers batch 0 again, so every step does the same work.  rpipe:
    # batches 0 and 1 are hashed here, before the timed region (the pipeline's fill).
    comm_prefetch_flag = comm_prefetch
    comm_prefetch = comm_prefetch and rf is not None
    rpl = pkg.distributed.ReplicatedPipeline(rf, batches, batch, fused_hash=rpipe) if comm_prefetch else None

    # Every timed insert asks for any_new, the reference's !found that drives EXPIRE
    # (ruby.rb:61-62): one pre-zeroed flag word per step, so no memset joins the step.
    flags = torch.zeros(len(batches), dtype=torch.int32, device=dev)
    fstep = [0]

    def any_new_ptr():
        i = fstep[0]
        fstep[0] = i + 1
        return flags[i % len(batches)].data_ptr()

    def insert(bt):
        ikb, iko = bt[0]
        if pipeline:
            f.insert_digests_dev(digs[step_no[0] % 2].data_ptr(), batch, d_any_new=any_new_ptr(), stream=sp)
        elif comm_prefetch:
            # the sizes of batch i+2 are all-gathered now, so step i+1's gather_start reads them
            # from pinned memory without waiting for the kernels in flight
            rpl.insert()
        elif rf is not None:
            rf.insert_many_dev(ikb, iko, batch)
        elif pf is None:
            f.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), batch, d_any_new=any_new_ptr(), stream=sp)
        else:
            pf.insert_many_dev(ikb, iko, batch)

    def include(bt):
        pkb, pko = bt[1]
        if pipeline:
            i = step_no[0]
            nkb, nko = batches[(i + 1) % len(batches)][0]
            f.include_hash_dev(pkb.data_ptr(), pko.data_ptr(), batch, out.data_ptr(), nkb.data_ptr(), nko.data_ptr(),
                               batch, digs[(i + 1) % 2].data_ptr(), stream=sp)
            step_no[0] = i + 1
        elif comm_prefetch:   # include? of batch i (rpipe: with batch i+2's SHA-1 fused in)
            rpl.include(out)
        elif rf is not None:
            out.copy_(rf.include_many_dev(pkb, pko, batch))
        elif pf is None:
            f.include_many_dev(pkb.data_ptr(), pko.data_ptr(), batch, out.data_ptr(), stream=sp)
        else:
            out.copy_(pf.include_many_dev(pkb, pko, batch))

    # Partitioned, comm_prefetch (sync-free exchange): step i routes and sends batch i+1's
    # inserts beside its own owner kernels (PartitionedFilter.insert_include_dev next_insert);
    # every step still applies all ranks' batch-i inserts before its include?.
    pf_prefetch = comm_prefetch_flag and pf is not None and overlap and pf.sync_free

    def part_step(i):
        (ikb, iko), (pkb, pko) = batches[i]
        nxt = (batches[(i + 1) % len(batches)][0] + (batch,)) if pf_prefetch else None
        out.copy_(pf.insert_include_dev(ikb, iko, batch, pkb, pko, batch, next_insert=nxt))

    for i, bt in enumerate(batches[:warmup]):
        if pf is None or not overlap:
            insert(bt)
            include(bt)
        else:
            part_step(i)
    prof = pf.engine.filter if pf is not None else f
    prof.profile(True)      # per-kernel HIP events, recorded on the launch stream inside the timed region
    prof.profile_read(reset=True)
    D.barrier()
    torch.cuda.synchronize()
    ev = []
    host_wait0 = rf.host_wait_s if rf is not None else 0.0
    t_start = time.perf_counter()
    for i, bt in enumerate(batches[warmup:], start=warmup):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(stream)
        if pf is None or not overlap:
            insert(bt)
            e[1].record(stream)
            include(bt)
        else:   # partitioned: one overlapped insert + include? step (same results)
            e[1].record(stream)
            part_step(i)
        e[2].record(stream)
        ev.append(e)
    torch.cuda.synchronize()
    D.barrier()
    wall = time.perf_counter() - t_start
    if rpl is not None:   # the wrap-around gather of batch 0 (comm_prefetch)
        rpl.drain()
        rf.sets_check()   # no region-set apply skipped a buffer or a region
    if pf_prefetch:   # the wrap-around route of batch 0 (already inserted: idempotent)
        pf.drain_prefetch()
    wall = D.max(wall)
    ins_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    inc_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    if pf is not None and overlap:   # the step is one overlapped unit: split it evenly for the per-op lines
        ins_ms = inc_ms = (ins_ms + inc_ms) / 2
    kernels = {name: {"ms": tot / cnt, "launches": cnt} for name, (tot, cnt) in prof.profile_read(reset=True).items()}
    prof.profile(False)
    plan = f.insert_plan(batch) if pf is None else {"binned": False, "scratch_bytes": 0}
    inc_binned = "bin_test" in kernels
    # sanity: the members (first half of the include? batch) must all be found
    got = out.cpu().numpy()
    assert got[: batch // 2].all(), "false negative in the include? batch"
    any_new_steps = int(flags[:fstep[0]].ne(0).sum().item())
    if fstep[0] and prefill == "random":   # 2^24 fresh keys into a half-empty filter flip bits
        assert any_new_steps == fstep[0], "an insert batch reported any_new = false"
    fp_rate = float(got[batch // 2:].mean())
    Lmean = float(batches[-1][1][1][-1].item()) / batch
    P = batch * k
    bitset = f.device_bytes
    # algorithmic bytes per launch of each kernel (SURVEY §8 d for the random-access kernels;
    # the binned insert's kernels by the arrays each one must read and write)
    E = 4 if (pf is None or pf.engine.offset_dtype == torch.int32) else 8   # routed offset bytes
    algo = {
        "bf_keys_kernel<INCLUDE>": batch * (Lmean + 8 + 1 + k * GRANULE),
        "bf_keys_kernel<INSERT>": batch * (Lmean + 8 + 2 * k * GRANULE),
        "bf_keys_kernel<INSERT_FLAGS>": batch * (Lmean + 8 + 2 * k * GRANULE + 1),
        # binned path (bf_binned.hip): keys in, probe arrays written / read once, the bitset
        # streamed once (read + write for insert, read for include?)
        "bin_front": batch * (Lmean + 8) + P * 4,
        # pipelined steps: the front pass reads 16 B of SHA-1 words per key; the include?
        # kernel also reads the next batch's keys and writes their words
        "bin_front_digest": batch * 16 + P * 4,
        "include_hash_kernel": batch * (Lmean + 8 + 1 + k * GRANULE) + batch * (Lmean + 8 + 16),
        "bin_front_keys": batch * (Lmean + 8) + P * 8 + batch,
        "bin_mid": P * 4 * 3,
        "bin_mid_keys": P * 8 * 3,
        "bin_apply": P * 4 + 2 * bitset,
        "bin_test": P * 8 + bitset,
        # partitioned (P = probes one rank sends, about what it receives): requester route,
        # owner-side sort of the routed offsets, direct shard ops, combine
        "route_front": batch * (Lmean + 8) + P * (E if E == 4 else 5),
        "route_front_slot": batch * (Lmean + 8) + P * ((E if E == 4 else 5) + 4),
        "route_win": batch * (Lmean + 8) + P * E,
        "route_win_slot": batch * (Lmean + 8) + P * (E + 4),
        "route_gather": P * ((E if E == 4 else 5) + E),
        "route_gather_slot": P * ((E if E == 4 else 5) + E + 8),
        "bin_front_offsets": P * (E + 4),
        "bin_front_offsets_keys": P * (E + 8),
        "shard_insert": P * 2 * GRANULE,
        "shard_test": P * (GRANULE + 1),
        "combine": P * 5 + batch,
    }
    for name, kt in kernels.items():
        if name in algo:
            kt["algo_bytes"] = algo[name]
            kt["GBps"] = algo[name] / (kt["ms"] / 1e3) / 1e9
    res = {
        "m": m, "k": k, "batch": batch, "mean_key_bytes": round(Lmean, 3), "pipelined": pipeline or rpipe,
        "wall_s": wall, "steps": steps,
        "keys_per_s": 2 * batch * D.world * steps / wall,
        "insert": {"op_ms": ins_ms, "keys_per_s": batch / (ins_ms / 1e3),
                   "path": "binned" if plan["binned"] else "direct",
                   "algo_bytes_per_key": (Lmean + 8 + 2 * bitset / batch) if plan["binned"]
                   else (Lmean + 8 + 2 * k * GRANULE),
                   # SURVEY §8(d)'s random-access model (L + 8 + 2kG) prices the direct insert;
                   # the binned insert streams the bitset once instead (L + 8 + 2 * bitset /
                   # batch), so only that model's fraction of 8 TB/s is given for it (the random
                   # model's would exceed 1 without any work skipped: VERDICT r04 weak 3)
                   "frac_random_model": None if plan["binned"] else
                   batch / (ins_ms / 1e3) * (Lmean + 8 + 2 * k * GRANULE) / HBM_PEAK,
                   "frac_streaming_model": batch / (ins_ms / 1e3) * (Lmean + 8 + 2 * bitset / batch) / HBM_PEAK
                   if plan["binned"] else None,
                   "roofline_model": "streaming (binned: the bitset read and written once per batch)"
                   if plan["binned"] else "random access (SURVEY §8 d: L + 8 + 2kG)"},
        "include": {"op_ms": inc_ms, "keys_per_s": batch / (inc_ms / 1e3),
                    "path": "binned" if inc_binned else "direct",
                    "algo_bytes_per_key": (Lmean + 8 + 1 + bitset / batch) if inc_binned
                    else (Lmean + 8 + 1 + k * GRANULE),
                    "observed_fp_rate": fp_rate},
        "kernels": kernels,
        "bitset_bytes": bitset,
        "any_new_requested": bool(fstep[0]), "any_new_steps": any_new_steps,
    }
    ib, io = to_host(*batches[0][0])
    pb, po = to_host(*batches[0][1])
    if want_host and pf is None:
        # PCIe-inclusive rate of the host-pointer entry points (pageable numpy keys + uint64
        # offsets in, answers out), after one warm-up call that sizes the pinned staging.
        # Median of 5 timed calls each (the box's host share is noisy); include? writes into a
        # caller-owned buffer, as the C ABI / Ruby FFI caller does (a fresh numpy result per call
        # adds its page faults: reported apart).
        torch.cuda.synchronize()
        f.insert_many(ib, io)
        ans = f.include_many(pb, po)
        out = np.empty(batch, np.uint8)

        def med(fn, reps=5):
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t)
            return sorted(ts)[reps // 2]

        t_ins = med(lambda: f.insert_many(ib, io))
        t_inc = med(lambda: f.include_many(pb, po, out=out))
        t_inc_fresh = med(lambda: f.include_many(pb, po), reps=3)
        assert np.array_equal(out, ans)
        res["host_api"] = {"insert_keys_per_s": batch / t_ins, "include_keys_per_s": batch / t_inc,
                           "include_fresh_result_keys_per_s": batch / t_inc_fresh,
                           "timing": "median of 5 calls (fresh-result include?: of 3)",
                           "pcie_bytes_per_key": float(io[-1]) / batch + 4,
                           "host_threads": int(os.environ.get("BFHIP_HOST_THREADS", "0")) or
                           min(16, usable_cores())}
    del batches
    if pf is not None:
        pf.close()
    else:
        f.close()
    res["mode"] = mode
    if rf is not None:
        res["replicated_insert_mode"] = rf.last_insert_mode
        # host time blocked on batch sizes inside the timed steps (pipelined: ~0)
        res["replicated_host_wait_ms_per_step"] = (rf.host_wait_s - host_wait0) / steps * 1e3
    return res, (ib, io, pb, po, host_bits, m, k)


# Per-rank models of the multi-GPU layouts, timed on this one GPU by tools/sim_rank.py (the kernels
# one rank runs per step; the exchange itself is not in them): the partitioned north-star filter
# at P = 8 (the driver's N = 8 layout), BASELINE configs[4] (200B@0.01 %, partitioned x 8) and
# configs[3] (10B@0.01 %, replicated x 8: one replica's step).  With no 8-GPU node the driver's
# own run is the only independent check of them.
MODEL_LEGS = {
    "model_P8_nstar": (["--shards", "8", "--chunks", "--config", "nstar", "--steps", "5"], "nstar", "partitioned"),
    "model_P8_200b": (["--shards", "8", "--chunks", "--config", "200b", "--steps", "5"], "200b", "partitioned"),
    "model_repl8_10b": (["--replicated", "8", "--config", "10b", "--gathered", "sets", "--fused-hash",
                         "--overlap-encode", "apply", "--steps", "3"], "10b", "replicated"),
}


def model_legs(names, single_ms: dict) -> dict:
    """Each model's per-rank step (partitioned: the kernels' sum — the stand-in receive copies
    are the exchange's job; replicated: the replica's wall time, every kernel of the step), its
    kernel breakdown, its PMC source and the predicted weak-scaling efficiency = the single-GPU
    step of the same filter (this run's line) / the per-rank step, before any exchange time."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("sim_rank", os.path.join(ROOT, "tools", "sim_rank.py"))
    sim = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sim)
    out = {}
    for name in names:
        argv, config, layout = MODEL_LEGS[name]
        t0 = time.time()
        r = sim.run(argv)
        torch.cuda.synchronize()
        per_rank = r["kernels_ms_sum"] if layout == "partitioned" else r["ms_per_step_compute"]
        one = single_ms.get(config)
        out[name] = {"layout": layout, "config": config, "world": 8, "argv": " ".join(argv),
                     "per_rank_ms": per_rank, "wall_ms_per_step": r["ms_per_step_compute"],
                     "single_gpu_ms_per_step": one,
                     "predicted_efficiency": one / per_rank if one else None,
                     "kernels": {kn: round(v, 4) for kn, v in r["kernels_ms_per_step"].items()},
                     "pmc": load_pmc(name), "model_s": round(time.time() - t0, 1),
                     "note": "one rank's compute per step on this GPU (tools/sim_rank.py); the all-to-all / "
                             "all-gather is not in it"}
        log("[%s] per-rank %.3f ms, single GPU %s ms" % (name, per_rank, one))
    return out


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cores() -> int:
    """CPUs this process can keep busy: its affinity mask, capped by the cgroup CPU quota
    (a gpurun box exposes all 256 CPUs of the host in the mask but grants one GPU's share,
    16, through cpu.max) and by OMP_NUM_THREADS when set."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            quota, period = fh.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def _time_oracle(orc, data, threads: int, budget_s: float):
    """Keys/s of the oracle's insert + include? over the first step's batches (2^20-key
    chunks, passed over again until ~budget_s of work is done) on `threads` OpenMP threads."""
    ib, io, pb, po, host_bits, m, k = data
    bits = host_bits.copy() if host_bits is not None else orc.new_bitset(m, k)
    done = 0
    n_total = len(io) - 1
    chunk = 1 << 20 if threads > 1 else 1 << 17
    i = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        j = min(i + chunk, n_total)
        orc.insert_many_omp(bits, m, k, ib, io[i:j + 1], threads)
        orc.include_many_omp(bits, m, k, pb, po[i:j + 1], threads)
        done += 2 * (j - i)
        i = j if j < n_total else 0
    dt = time.perf_counter() - t0
    return done / dt, done, dt


def cpu_baseline(data, budget_s: float = 10.0):
    """The oracle (oracle/bf_oracle.c: the same SHA-1, offsets and byte-order bitset, OpenMP)
    on the host, on a bounded sample of the same workload: all the cores this process may
    use (usable_cores(): a gpurun box grants one GPU 16 of its host's cores) and one core.  The
    reference's own drivers need ruby + redis-server, probed here and recorded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O   # the checker, here the timed CPU baseline ("port")
    orc = O.COracle()
    cores = usable_cores()
    v_all, d_all, t_all = _time_oracle(orc, data, cores, budget_s)
    v_one, d_one, t_one = _time_oracle(orc, data, 1, budget_s)
    import shutil
    tools = {t: shutil.which(t) for t in ("ruby", "redis-server", "lua")}
    n_total = len(data[1]) - 1
    return {"value": v_all, "unit": "keys/s", "cores": cores, "kind": "port",
            "single_core": {"value": v_one, "cores": 1,
                            "sample": "%d insert + %d include? keys, %.1f s" % (d_one // 2, d_one // 2, t_one)},
            "cpu_model": cpu_model(), "machine_cpus": os.cpu_count(),
            "sample": "%d insert + %d include? keys (the first step's %d-key batches, repeated) on the same "
                      "prefilled filter, oracle/bf_oracle.c with OpenMP on %d threads, %.1f s"
                      % (d_all // 2, d_all // 2, n_total, cores, t_all),
            "reference_drivers": {"tools": tools, "timed": all(tools[t] for t in ("ruby", "redis-server")),
                                  "note": "the reference ruby/lua drivers (bf_100_000_flat.rb shape) need ruby + "
                                          "redis-server; absent on this box, so only their published "
                                          "README.md:80-95 numbers are quoted"}}


def _w8_words(rng, count: int):
    """bf_10_000.rb:8-11 rand_word: 8 distinct letters of a..z, sampled in order."""
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8)
    return [letters[rng.permutation(26)[:8]].tobytes().decode() for _ in range(count)]


def reference_shapes(pkg, per_key_ops: int = 20000, words_n: int = 10000, flat_items: int = 100000,
                     big_keys: int = 1 << 22):
    """The reference's own benchmark loops, run through the Python facade
    (``Bloomfilter(driver: 'hip' | 'hip-lua' | 'hip-test')``) against the in-process FakeRedis,
    write-through sync on (every insert that flips a bit SETRANGEs the changed 64 KiB blocks):

    * ``bf_10_000`` — BASELINE configs[0], benchmark/bf_10_000.rb:20-43: 10,000 W8 words, per
      key include? (counted against a visited set) then insert, for each hip driver;
    * ``flat`` — benchmark/bf_100_000_flat.rb:8-24 (README.md:80-95 at 1M): a 100,000-item
      filter, ``per_key_ops`` per-key inserts of rand(items) then as many include?s, and the
      whole 100,000 of each as one batched call;
    * ``100m_sync`` — BASELINE configs[2]: the 100M@0.1 % filter (180 MB string), one
      insert_many of 2^22 keys with write-through (the whole string changes, so it is all
      SETRANGEd in 8 MiB chunks), then include_many of 2^22 keys.

    Per-key ops pay Python + ctypes + one host-pointer round trip each; the reference pays a
    Redis round trip per op (~160-230 us, README.md:86-93)."""
    fr = pkg.fakeredis
    rng = np.random.default_rng(SEED)
    out = {}
    words = _w8_words(rng, words_n)
    for drv in ("hip", "hip-lua", "hip-test"):
        bf = pkg.Bloomfilter(size=words_n, error_rate=0.01, key_name="bloom-filter-bench-" + drv, driver=drv,
                             redis=fr.FakeRedis())
        bf.clear()
        error, first, visited = 0, 0, set()
        t0 = time.perf_counter()
        for i, w in enumerate(words):
            if bf.include(w) != (w in visited):
                error += 1
                if error == 1:
                    first = i
            visited.add(w)
            bf.insert(w)
        dt = time.perf_counter() - t0
        out.setdefault("bf_10_000", {})[drv] = {
            "ops_per_s": 2 * len(words) / dt, "us_per_op": dt / (2 * len(words)) * 1e6,
            "errors": error, "first_error_at": first, "bits": bf.options["bits"], "hashes": bf.options["hashes"],
            "redis_string_sha1": hashlib.sha1(bf.redis.get("bloom-filter-bench-" + drv) or b"").hexdigest()
            if drv != "hip-lua" else None}
        bf.driver.close()
    items = flat_items
    vals = rng.integers(0, items, size=items)
    for drv in ("hip", "hip-lua"):
        bf = pkg.Bloomfilter(size=items, error_rate=0.01, key_name="bloom-filter-bench-flat-" + drv, driver=drv,
                             redis=fr.FakeRedis())
        bf.clear()
        sample = [int(v) for v in vals[:per_key_ops]]
        t0 = time.perf_counter()
        for v in sample:
            bf.insert(v)
        t_ins = time.perf_counter() - t0
        t0 = time.perf_counter()
        for v in sample:
            bf.include(v)
        t_inc = time.perf_counter() - t0
        bf.clear()
        t0 = time.perf_counter()
        bf.insert_many(vals)
        b_ins = time.perf_counter() - t0
        t0 = time.perf_counter()
        hits = bf.include_many(vals)
        b_inc = time.perf_counter() - t0
        assert bool(np.all(hits)), "flat: an inserted key answered false"
        out.setdefault("flat", {})[drv] = {
            "per_key_insert_ops_per_s": len(sample) / t_ins, "per_key_include_ops_per_s": len(sample) / t_inc,
            "per_key_sample": len(sample),
            "batched_insert_keys_per_s": items / b_ins, "batched_include_keys_per_s": items / b_inc}
        bf.driver.close()
    n_items, err = CONFIGS["100m"][:2]
    bf = pkg.Bloomfilter(size=n_items, error_rate=err, key_name="bench-100m", driver="hip", redis=fr.FakeRedis())
    drv, r = bf.driver, bf.redis
    ikeys = rng.integers(0, 1 << 62, size=big_keys)
    half = big_keys // 2
    qkeys = np.concatenate([ikeys[:half], rng.integers(0, 1 << 62, size=big_keys - half)])
    t0 = time.perf_counter()
    ib, io = pkg.keys.pack(ikeys)
    t_pack = time.perf_counter() - t0
    qb, qo = pkg.keys.pack(qkeys)
    # warm-up: a quarter-size call of each op (the host path's pinned staging is sized by its
    # chunks, so the full-size calls below reuse it), then the first full insert, whose any_new
    # must be true; insert / include? are the median of 5 full-size calls (a repeated insert
    # does the same device work: the binned apply streams the whole 180 MB bitset regardless)
    w = min(len(ikeys) // 4, 1 << 20)
    drv.filter.insert_many(ib[: int(io[w])], io[: w + 1], any_new=True)
    drv.filter.include_many(qb[: int(qo[w])], qo[: w + 1])
    t0 = time.perf_counter()
    any_new, _ = drv.filter.insert_many(ib, io, any_new=True)
    t_first = time.perf_counter() - t0

    def med(fn, reps=5):
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        return sorted(ts)[reps // 2], ts

    t_ins, ins_all = med(lambda: drv.filter.insert_many(ib, io, any_new=True))
    ranges, slen = drv.filter.dirty_ranges(clear=False)
    t0 = time.perf_counter()
    for off, ln in ranges:   # the device side of the sync alone: D2H of the changed ranges
        for c in range(off, off + ln, drv.chunk_bytes):
            drv.filter.export_range(c, min(drv.chunk_bytes, off + ln - c))
    t_export = time.perf_counter() - t0
    t0 = time.perf_counter()
    sent = drv.flush()   # dirty ranges -> export -> SETRANGE into the FakeRedis string
    t_sync = time.perf_counter() - t0
    hits = np.empty(len(qkeys), np.uint8)
    t_inc, inc_all = med(lambda: drv.filter.include_many(qb, qo, out=hits))
    assert any_new and bool(np.all(hits[:half])), "100m_sync: an inserted key answered false"
    # what bounds these calls: the host side copies every key byte and offset into pinned
    # staging (16 threads) before the H2D; the same bytes copied by 16 host threads here
    host_bytes = int(io[-1]) + 4 * (len(ikeys) + 1)
    src = np.asarray(ib).view(np.uint8)[: int(io[-1])]
    dst = np.empty_like(src)
    from concurrent.futures import ThreadPoolExecutor
    cuts = np.linspace(0, len(src), 17).astype(np.int64)

    def pcopy():
        with ThreadPoolExecutor(16) as ex:
            list(ex.map(lambda a: np.copyto(dst[cuts[a]:cuts[a + 1]], src[cuts[a]:cuts[a + 1]]), range(16)))

    pcopy()
    t_copy, _ = med(pcopy, 3)
    assert r.get("bench-100m") == drv.to_redis_string(), "100m_sync: Redis string differs from the device"
    out["100m_sync"] = {"bits": bf.options["bits"], "hashes": bf.options["hashes"], "keys": len(ikeys),
                        "host_pack_keys_per_s": len(ikeys) / t_pack,
                        "insert_keys_per_s": len(ikeys) / t_ins, "include_keys_per_s": len(qkeys) / t_inc,
                        "timing": "median of 5 full-size calls after warm-up (include? into a caller-owned "
                                  "answer buffer, as the Ruby FFI driver's)",
                        "insert_ms_calls": [round(x * 1e3, 2) for x in ins_all],
                        "include_ms_calls": [round(x * 1e3, 2) for x in inc_all],
                        "first_insert_keys_per_s": len(ikeys) / t_first,
                        "host_bytes_per_call": host_bytes,
                        "host_bytes_GBps_insert": host_bytes / t_ins / 1e9,
                        "host_memcpy_GBps_16_threads": len(src) / t_copy / 1e9,
                        "redis_string_bytes": slen, "synced_bytes": sent,
                        "export_GBps": sent / t_export / 1e9, "sync_s": t_sync,
                        "sync_GBps": sent / t_sync / 1e9,
                        "note": "insert/include: the host-pointer ABI (PCIe-inclusive, keys packed beforehand); "
                                "export: D2H of the dirty ranges; sync: dirty ranges -> export -> SETRANGE "
                                "into the in-process FakeRedis string (8 MiB requests)"}
    drv.close()
    out["redis"] = "in-process FakeRedis (redis-bloomfilter_amd/fakeredis.py); no redis-server on the box"
    return out


def load_traffic(workload: str, kernel: str):
    """(PMC-measured HBM bytes per launch of `kernel`, the PMC summary they come from)
    (profiles/pmc_traffic.json, tools/pmc_summary.py), or (None, None)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            doc = json.load(fh)
    except (OSError, ValueError):
        return None, None
    rec = (doc.get(workload) or {}).get(kernel)
    if not isinstance(rec, dict) or rec.get("hbm_bytes_per_launch") is None:
        return None, None
    return rec["hbm_bytes_per_launch"], doc.get("source")


# every workload's counters from the round's final tree, one tag (tools/pmc_finalize.py;
# tests/test_profiles_tagged.py checks the tag across these, pmc_traffic.json and the rocprof means)
PMC_TAG = "r06ac"
PMC_FILES = {w: "pmc_%s_%s.json" % (PMC_TAG, w) for w in ("nstar", "1m", "1m_big", "100m", "10b", "200b", "lua_1m",
                                                          "model_P8_nstar", "model_P8_200b", "model_repl8_10b")}
# rocprofv3 --kernel-trace --stats of the bench command on the round's final tree
# (tools/rocprof_means.py over profiles/<tag>_kernel_stats.csv): each kernel's mean launch
ROCPROF_MEANS = "rocprof_means.json"


def load_rocprof_mean(workload: str, kernel: str):
    """(mean ms, source) of `kernel` from the committed rocprof summary, or (None, None)."""
    try:
        with open(os.path.join(ROOT, "profiles", ROCPROF_MEANS)) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None, None
    rec = (t.get(workload) or {}).get(kernel)
    return (rec, t.get("source")) if rec else (None, None)


def load_pmc(workload: str):
    """VALU and traffic counters per kernel from the committed PMC passes of this workload
    (tools/pmc_passes.sh + tools/pmc_summary.py; rocprofv3 cannot run inside the bench
    itself): valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)."""
    name = PMC_FILES.get(workload)
    if not name:
        return None
    try:
        with open(os.path.join(ROOT, "profiles", name)) as fh:
            t = json.load(fh).get(workload) or {}
    except (OSError, ValueError):
        return None
    keep = ("valu_busy", "valu_lane_insts_per_key", "hbm_bytes_per_launch", "profiled_ms_mean", "frac_wait_any",
            "frac_wait_inst_any", "frac_active_inst_any", "lds_bank_conflict_frac")
    return {"source": "profiles/" + name,
            "kernels": {kn: {x: rec.get(x) for x in keep} for kn, rec in t.items() if isinstance(rec, dict)}}


def _free_port() -> int:
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(gpus: int, argv, json_out) -> int:
    """``python bench.py --gpus N`` started without a launcher (no WORLD_SIZE): start the N
    ranks as ONE child ``torch.distributed.run`` (a fresh process, started before this one
    touches the GPU — no exec), relay rank 0's JSON line, and return the child's exit code.
    The ranks see WORLD_SIZE = N, so the line's n_gpus is N or the run fails."""
    import subprocess
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", BFBENCH_SELF_LAUNCHED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    log("bench: --gpus %d without WORLD_SIZE: launching %d ranks (%s)" % (gpus, gpus, " ".join(cmd[1:6])))
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    relayed = 0
    for ln in proc.stdout:   # rank 0's JSON line; anything else a library printed goes to stderr
        if ln.lstrip().startswith("{"):
            print(ln.rstrip("\n"), file=json_out, flush=True)
            relayed += 1
        else:
            sys.stderr.write(ln)
    rc = proc.wait()
    if rc == 0 and relayed != 1:
        log("bench: the %d-rank run printed %d JSON lines, expected 1" % (gpus, relayed))
        return 3
    return rc


def check_world(gpus: int) -> None:
    """A launcher's world size must be the --gpus asked for: a mismatch would report an N-GPU
    number for another N."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None and int(world) != gpus:
        log("bench: --gpus %d but WORLD_SIZE=%s: refusing to report a %s-rank run as %d GPUs"
            % (gpus, world, world, gpus))
        sys.exit(2)


def launch_check(D: "Dist", json_out) -> None:
    """--launch-check: the process group as bench.py builds it, then rank 0 reports the world
    it saw and exits (no filter, no GPU work): what the CPU tests check of the N-rank launch."""
    seen = dist.get_world_size() if dist.is_initialized() else 1
    if D.rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": D.world, "world_size_seen": seen,
                          "backend": D.backend,
                          "self_launched": os.environ.get("BFBENCH_SELF_LAUNCHED") == "1"}),
              file=json_out, flush=True)
    D.close()


def main():
    # Libraries (RCCL's version banner, HIP) may write to stdout; the contract is ONE JSON
    # line there, so fd 1 goes to stderr for the run and the JSON to the original stdout.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="nstar", choices=sorted(CONFIGS))
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--secondary", default="1m,1m_big,100m,10b,200b,lua_1m",
                    help="comma list of the secondary workloads (1-GPU runs): configs and lua_1m")
    ap.add_argument("--models", default=",".join(MODEL_LEGS),
                    help="comma list of the per-rank multi-GPU models timed on this GPU (tools/sim_rank.py), "
                         "'' for none: %s" % ", ".join(MODEL_LEGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-api", action="store_true", help="skip the PCIe-inclusive host-API timing")
    ap.add_argument("--no-reference-shapes", action="store_true",
                    help="skip the reference benchmark loops through the facade (bf_10_000.rb, "
                         "bf_100_000_flat.rb, 100M with Redis sync)")
    ap.add_argument("--mode", default="auto", choices=["auto", "single", "partitioned", "replicated"],
                    help="auto: single GPU at N=1, replicated at N=2 (filter fits one GPU), partitioned from N=4")
    ap.add_argument("--no-overlap", action="store_true",
                    help="partitioned: run insert then include? as separate calls (no exchange overlap)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="single GPU: 1 = pipelined steps (next insert batch hashed inside the include? "
                         "kernel, inserted from its SHA-1 words), 0 = plain insert_many + include_many")
    ap.add_argument("--comm-prefetch", type=int, default=1,
                    help="1 = exchange the next step's insert batch during this step (replicated: gather "
                         "its keys, then insert every rank's batch as one insert; partitioned: route and "
                         "send its probes beside this step's owner kernels); 0 = within the step")
    ap.add_argument("--replicated-insert", default="auto", choices=["auto", "gather", "or", "digests", "sets"],
                    help="replicated layout: what every rank's insert batch travels as (ReplicatedFilter "
                         "insert_mode); auto: the per-config choice REPLICATED_INSERT, else by size")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL) is the measured path; gloo rehearses N > 1 with host-staged "
                         "exchanges, several ranks per GPU allowed (not a performance number)")
    ap.add_argument("--launch-check", action="store_true",
                    help="build the process group, print the world size rank 0 saw, exit (no GPU work)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        json_out.flush()
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], json_out))
    check_world(args.gpus)

    D = Dist(need_group=(args.mode in ("partitioned", "replicated")), backend=args.dist_backend,
             no_device=args.launch_check)
    if args.launch_check:
        return launch_check(D, json_out)
    world_seen = dist.get_world_size() if dist.is_initialized() else 1
    if world_seen != args.gpus:
        log("bench: the process group has %d ranks, --gpus %d" % (world_seen, args.gpus))
        sys.exit(2)
    pkg = pkgload.load()
    main_res, data = time_config(pkg, D, args.config, args.steps, args.warmup, want_host=(D.world == 1 and not args.no_host_api),
                                  mode=args.mode, overlap=not args.no_overlap, pipeline=bool(args.pipeline),
                                  comm_prefetch=bool(args.comm_prefetch), replicated_insert=args.replicated_insert)
    secondary = {}
    if D.world == 1 and not args.no_secondary:
        # 1m_big: the L2-resident 1M@1 % filter at 2^24-key batches (hash-bound; 1m's 2^20-key
        # batches are launch- and latency-bound)
        # every secondary runs the step `--config <name>` runs (pipelined unless --pipeline 0),
        # so the driver's line carries the same numbers a --config run reports
        for name in [x for x in args.secondary.split(",") if x]:
            if name == "lua_1m":   # SURVEY §8 f1, the Lua layout on the device
                secondary[name] = lua_config(pkg, D)
            elif name != args.config:
                r, _ = time_config(pkg, D, name, max(3, args.steps // 2), 1, pipeline=bool(args.pipeline))
                secondary[name] = {"keys_per_s": r["keys_per_s"], "pipelined": r["pipelined"],
                                   "ms_per_step": r["wall_s"] / r["steps"] * 1e3,
                                   "insert_keys_per_s": r["insert"]["keys_per_s"],
                                   "include_keys_per_s": r["include"]["keys_per_s"],
                                   "m": r["m"], "k": r["k"], "batch": r["batch"],
                                   "kernels": {kn: round(v["ms"], 4) for kn, v in r["kernels"].items()},
                                   "pmc": load_pmc(name)}
    models = None
    if D.world == 1 and args.models and not args.no_secondary:
        single = {name: r["ms_per_step"] for name, r in secondary.items() if "ms_per_step" in r}
        single[args.config] = main_res["wall_s"] / args.steps * 1e3
        models = model_legs([x for x in args.models.split(",") if x and x != "none"], single)
    shapes = None
    if D.world == 1 and not args.no_reference_shapes:
        shapes = reference_shapes(pkg)
    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(data)
    D.close()
    if D.rank != 0:
        return

    ins, inc = main_res["insert"], main_res["include"]
    # dominant kernel: the largest total time per step among the kernels the ops launched
    kern = main_res["kernels"]
    dom_name = max(kern, key=lambda nm: kern[nm]["ms"] * kern[nm]["launches"])
    dom = kern[dom_name]
    achieved = dom["algo_bytes"] / (dom["ms"] / 1e3) if "algo_bytes" in dom else None
    rp_ms, rp_src = load_rocprof_mean(args.config, dom_name)
    traffic, traffic_src = load_traffic(args.config, dom_name)
    n, p, batch, _ = CONFIGS[args.config]
    fills = None
    if dom_name in ("include_hash_kernel", "bf_keys_kernel<INCLUDE>"):
        # the direct include?'s random line fills per key: members probe all k offsets,
        # non-members stop at the first 0 bit (bit density d = fp^(1/k) from the batch's
        # observed false-positive rate), half of each in the batch
        kk, fp = main_res["k"], inc["observed_fp_rate"]
        d = fp ** (1.0 / kk) if fp > 0 else 0.0
        per_key = 0.5 * kk + 0.5 * ((1 - fp) / (1 - d) if d < 1 else kk)
        rate = batch * per_key / (dom["ms"] / 1e3)
        ceil, ceil_src = fill_ceiling(main_res["bitset_bytes"])
        fills = {"fills_per_key": per_key, "bit_density": d, "fills_per_s": rate, "ceiling_fills_per_s": ceil,
                 "frac": rate / ceil, "ceiling_source": ceil_src}
    line = {
        "metric": "keys/sec (insert, include?) per GPU and whole node; % of HBM random-access roofline",
        "value": main_res["keys_per_s"],
        "unit": "keys/s",
        "n_gpus": D.world,
        # the process group's own size (RCCL communicator under nccl) and who started the ranks
        "world_size_seen": world_seen,
        "launcher": ("bench.py --gpus %d (one torch.distributed.run child)" % args.gpus
                     if os.environ.get("BFBENCH_SELF_LAUNCHED") == "1" else
                     "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ or D.world > 1 else "single process"),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main_res["wall_s"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: decimal-string keys of seeded uniform ints (bf_100_000_flat.rb shape); "
                "filter prefilled to 50% random bit density",
        "config": {"workload": "%s: %d keys @ %g error, m=%d bits, k=%d, batch=%d keys insert_many + %d keys "
                               "include_many? per step (50%% members)" % (args.config, n, p, main_res["m"],
                                                                          main_res["k"], batch, batch),
                   "global_batch": 2 * batch * D.world,
                   "parallelism": {"partitioned": "partitioned x%d (block-cyclic 2^20-bit blocks; per-rank key "
                                                  "batches routed to owner GPUs, grouped RCCL send/recv%s)"
                                                  % (D.world, "; the next step's inserts routed and sent during "
                                                     "this step" if args.comm_prefetch else ""),
                                   "replicated": "replicated x%d (include? local; every rank's insert batch "
                                                 "all-gathered over RCCL as keys, SHA-1 words or region sets "
                                                 "(sorted once by its own rank) and applied by every replica, or "
                                                 "own batch + OR-all-reduce of the bitset when that moves fewer "
                                                 "bytes: %s%s)"
                                                 % (D.world, main_res.get("replicated_insert_mode"),
                                                    "; the next step's batches gathered during this step"
                                                    if args.comm_prefetch else ""),
                                   "single": "single GPU"}[main_res["mode"]]
                   + ("" if args.dist_backend == "nccl" else
                      " [REHEARSAL over gloo, host-staged exchanges, %d GPU(s) shared: not a "
                      "performance number]" % max(torch.cuda.device_count(), 1))},
        "roofline": {"bound": "hbm", "kernel": dom_name,
                     "achieved": achieved / 1e9 if achieved else None, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK if achieved else None,
                     "traffic": traffic, "traffic_source": traffic_src,
                     # the PMC-measured fabric bytes per launch over the same launch time: what
                     # the kernel actually moves (128 B line fills; SURVEY's 64 B granule model
                     # undercounts them and overcounts the early exit's skipped probes)
                     "traffic_GBps": traffic / (dom["ms"] / 1e3) / 1e9 if traffic else None,
                     "traffic_frac": traffic / (dom["ms"] / 1e3) / HBM_PEAK if traffic else None,
                     "algo_bytes": dom.get("algo_bytes"), "keys_per_launch": batch,
                     # the include? kernel's own bound: random 128-B line fills per second
                     # against the measured random-fill ceiling of this chip
                     "random_fill": fills,
                     "kernel_ms": dom["ms"], "timing": "HIP events on the launch stream around each kernel, "
                                                       "inside the timed region (bf_profile)",
                     # the same fraction from the committed rocprofv3 --stats mean of this kernel
                     "kernel_ms_rocprof": rp_ms, "rocprof_source": rp_src,
                     "frac_rocprof": (dom["algo_bytes"] / (rp_ms / 1e3) / HBM_PEAK)
                     if rp_ms and "algo_bytes" in dom else None},
        "pmc": load_pmc(args.config),
        "cpu_baseline": cpu,
        "ops": {"insert": ins, "include": inc},
        "kernels": kern,
        "host_api": main_res.get("host_api"),
        "replicated_host_wait_ms_per_step": main_res.get("replicated_host_wait_ms_per_step"),
        "secondary": secondary or None,
        "multi_gpu_models": models,
        "reference_shapes": shapes,
        "reference_published_keys_per_s": {"ruby_insert": 5103, "ruby_include": 4322,
                                           "lua_insert": 6235, "lua_include": 5712,
                                           "source": "reference README.md:80-95, 1M items, hardware unstated"},
    }
    print(json.dumps(line), file=json_out, flush=True)


if __name__ == "__main__":
    main()
