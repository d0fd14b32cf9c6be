#!/usr/bin/env python3
"""Diagnostic: the sync-free exchange at RCCL world size 1, step by step, with every device
buffer the next kernel will index validated on the host first (so a bad index is reported
instead of launched).  Prints one line per step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
D = pkg.distributed


def say(*a):
    print(*a, flush=True)


def check_live(name, buf, counts, cap, limit, nwin, stride=1, col=0):
    c = counts.reshape(-1).cpu().numpy()
    b = buf.cpu().numpy()
    for w in range(nwin):
        live = int(c[w * stride + col])
        if live > cap:
            say("  %s window %d overflowed (%d > %d): skipped" % (name, w, live, cap))
            continue
        seg = b[w * cap: w * cap + live].astype(np.int64) & 0xFFFFFFFF
        if live and seg.max() >= limit:
            raise SystemExit("%s window %d: entry %d >= %d" % (name, w, int(seg.max()), limit))


def run(m, k, b, n_ins, n_inc, cap_sf=None):
    f = D.PartitionedFilter(m, k, block_log2=b)
    if cap_sf is not None:
        f._cap_sf = lambda n: cap_sf
    e, P, nh = f.engine, f.P, f.engine.nh
    say("m=%d k=%d b=%d nh=%d local_bits=%d cap_sf=%s" % (m, k, b, nh, e.filter.local_bits, cap_sf))
    keys = ["k%d" % i for i in range(n_ins)]
    probe = keys[: n_inc // 2] + ["x%d" % i for i in range(n_inc - n_inc // 2)]
    kb, ko, n = D._device_batch(keys, f.device)
    st = f._sf_start(kb, ko, n, want_slot=False)
    torch.cuda.synchronize()
    say(" insert routed: counts", st["counts"].cpu().tolist(), "cap", st["cap"], "rmsg", st["rmsg"].shape)
    f._sf_flag(st)
    torch.cuda.synchronize()
    say(" rmsg", st["rmsg"].cpu().tolist())
    lim = 1 << 32
    for h in range(nh):
        check_live("recv h=%d" % h, st["recv"][h * P * st["cap"]:(h + 1) * P * st["cap"]], st["rmsg"], st["cap"], lim, P,
                   nh + 1, h)
    f._sf_insert(st)
    torch.cuda.synchronize()
    say(" insert applied; overflowed:", f._sf_overflowed(st))
    qb, qo, nq = D._device_batch(probe, f.device)
    st = f._sf_start(qb, qo, nq, want_slot=True)
    f._sf_flag(st)
    torch.cuda.synchronize()
    say(" include routed: counts", st["counts"].cpu().tolist())
    check_live("slot", st["slot"], st["counts"], st["cap"], nq, P * nh)
    out = f._sf_answer(st)
    torch.cuda.synchronize()
    say(" include answered: hits", int(out.sum().item()), "of", nq, "overflowed:", f._sf_overflowed(st))
    f.close()


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    run(9585058, 6, 16, 50_000, 40_000)
    run(9585058, 6, 16, 50_000, 40_000, cap_sf=12288)
    run(9585058377, 6, 20, 50_000, 40_000)
    dist.destroy_process_group()
    say("SF_PROBE_OK")


if __name__ == "__main__" and not os.environ.get("SF_WORLD1"):
    main()


def world1_sequence():
    """tests/test_gpu_distributed.py::test_torch_distributed_world1's PartitionedFilter steps,
    with a synchronize + print after each (no kernel serialization)."""
    m, k = 9585058, 6
    keys = ["k%d" % i for i in range(50_000)]
    probe = keys[:20_000] + ["x%d" % i for i in range(20_000)]
    for cls, kw in ((D.PartitionedFilter, {"block_log2": 16}), (D.ReplicatedFilter, {}),
                    (D.ReplicatedFilter, {"insert_mode": "or"})):
        f = cls(m, k, **kw)
        f.insert_many(keys)
        torch.cuda.synchronize()
        say(" %s %s insert ok" % (cls.__name__, kw))
        got = f.include_many(probe)
        torch.cuda.synchronize()
        say(" include ok", int(got.sum()))
        s = f.export_redis()
        say(" export ok", len(s))
        f.close()
    for kw, cap in (({}, None), ({"windows": False}, None), ({"sync_free": False}, 5), ({}, "sf"),
                    ({"pack_answers": False}, None), ({"pack_answers": False, "sync_free": False}, None)):
        f = D.PartitionedFilter(m, k, block_log2=16, **kw)
        if cap == "sf":
            f._cap_sf = lambda n: f.WINDOW_ALIGN
        elif cap is not None:
            f._cap = lambda n, c=cap: c
        got = f.insert_include(keys, probe)
        torch.cuda.synchronize()
        say(" insert_include %s %s ok: hits %d replays %d overflows %d" % (kw, cap, int(got.sum()), f.replays,
                                                                          f.window_overflows))
        f.close()
    m = 9585058377
    for kw in ({}, {"windows": False}):
        f = D.PartitionedFilter(m, k, block_log2=20, **kw)
        got = f.insert_include(keys, probe)
        torch.cuda.synchronize()
        say(" 1.2 GB insert_include %s ok: hits %d" % (kw, int(got.sum())))
        f.close()
    say("WORLD1_OK")


if __name__ == "__main__" and os.environ.get("SF_WORLD1"):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29612")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    world1_sequence()
    dist.destroy_process_group()
