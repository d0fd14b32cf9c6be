#!/usr/bin/env python3
"""Per-rank compute of the partitioned filter at P shards, simulated on ONE GPU.

    python tools/sim_rank.py [--shards 8] [--config nstar] [--steps 5]

Builds shard 0 of a P-way partitioned north-star filter (the largest shard) and runs,
per step, the kernels one rank runs at world size P: route its 2^24-key insert batch,
apply a received batch of the same size to its shard, route its include? batch, test
a received batch, combine.  The received batches are this rank's own routed probes (in
a balanced run every rank receives about as many as it sends; every owner-local offset
is valid on shard 0, the largest).  No collective runs: the all-to-all time is not in
these numbers.  Prints one JSON line with per-kernel means (bf_profile).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402


def main():
    print(json.dumps(run(sys.argv[1:])))


def run(argv) -> dict:
    """The model for one command line (the CLI's flags); returns its JSON line as a dict.
    bench.py calls this for its per-rank model legs (model_P8_nstar, model_P8_200b,
    model_repl8_10b)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--config", default="nstar", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--windows", action="store_true",
                    help="route through bf_route_windows_dev (window send buffer, no gather pass); "
                         "a device copy of the windows stands in for the receive")
    ap.add_argument("--sync-free", action="store_true",
                    help="the default exchange's compute: whole windows of cap_sf entries, device-side "
                         "counts, windowed owner ops, packed answers (PartitionedFilter._sf_*); the "
                         "received windows are this rank's own (nh == 1 configs)")
    ap.add_argument("--chunks", action="store_true",
                    help="the sync-free exchange with chunked windows (bf_route_chunks_dev: the route sorts "
                         "each window's runs by owner superbin and writes a directory, the owner skips its "
                         "sort pass; the combine gathers per route tile); the received windows are this "
                         "rank's own, permuted into the receive layout (any nh)")
    ap.add_argument("--replicated", type=int, default=0,
                    help="R > 0: one replica's step of the replicated layout at world size R (BASELINE "
                         "configs[3]): ONE merged insert of every rank's batch (R x batch keys) into the whole "
                         "filter, then this rank's include? batch")
    ap.add_argument("--gathered", default="keys", choices=["keys", "digests", "sets"],
                    help="replicated: what travels — key bytes (every replica hashes every batch: "
                         "ReplicatedFilter), 16-B SHA-1 words (each key hashed once, by its own rank), or "
                         "region sets (each batch hashed, sorted and encoded once, by its own rank; every "
                         "replica ORs all R ranks' sets in without sorting)")
    ap.add_argument("--fused-hash", action="store_true",
                    help="--replicated --gathered sets: the own batch's SHA-1 words come out of the previous "
                         "step's include? kernel (bf_include_hash_dev) and the encode starts from them "
                         "(bench.py's pipelined replicated step)")
    ap.add_argument("--overlap-encode", default="", choices=["", "apply", "include"],
                    help="--replicated --gathered sets --fused-hash: the NEXT step's own encode runs on a second "
                         "stream (a second handle) from the start of this step's apply, or of its include?; "
                         "read the wall time")
    ap.add_argument("--main-priority", action="store_true",
                    help="--overlap-encode: the main step on a high-priority stream, the side encode at normal "
                         "priority")
    ap.add_argument("--fused-encode", action="store_true",
                    help="--replicated --gathered sets --fused-hash: this step's sets applied and the next batch's "
                         "own set encoded by one kernel (bf_insert_encode_region_sets_dev)")
    ap.add_argument("--side-priority", action="store_true",
                    help="--overlap-encode: the side encode on a high-priority stream")
    ap.add_argument("--dig", action="store_true",
                    help="--chunks: route the include? batch from SHA-1 words that the previous step's owner "
                         "test hashed between its probe rounds (bf_shard_test_chunks_hash_dev + "
                         "bf_route_chunks_digests_dev)")
    ap.add_argument("--dig-side", action="store_true",
                    help="--chunks --dig, but the next include? batch is hashed by bf_hash_many_dev on a second "
                         "stream (a second handle) beside the owner test, not inside it; read the wall time")
    ap.add_argument("--fused-dig", action="store_true",
                    help="--chunks (one owner pass): that pass also hashes the next step's include? batch "
                         "(bf_shard_insert_test_chunks_packed_dev with n_next), which the next step routes from "
                         "its words")
    ap.add_argument("--hash-split", dest="hash_split", action="store_true", default=True,
                    help="--chunks (default, as PartitionedFilter): each route as two kernels, the keys' SHA-1 "
                         "(bf_hash_many_dev, full occupancy) then the route from the words "
                         "(bf_route_chunks_digests_dev)")
    ap.add_argument("--no-hash-split", dest="hash_split", action="store_false",
                    help="--chunks: the route hashes the keys itself (the round-5 form)")
    ap.add_argument("--separate", action="store_true",
                    help="--chunks: the owner's insert and include? as two calls (shard_insert_chunks, then "
                         "shard_test_chunks_packed) instead of one pass over the shard")
    ap.add_argument("--packed-bytes", action="store_true",
                    help="--chunks: the owner test writes answer bytes and a pack pass makes the bits (the "
                         "round-5 form) instead of bf_shard_test_chunks_packed_dev")
    ap.add_argument("--no-prefill", action="store_true",
                    help="partitioned: start from an empty shard (default: 50 %% random bit density, as "
                         "bench.py prefills every rank's shard; the owner test stores an answer per 0-probe)")
    ap.add_argument("--overlap", action="store_true",
                    help="--chunks: route the NEXT step's insert batch on a second stream while this step's "
                         "owner kernels run (what PartitionedFilter's next_insert prefetch would do on a side "
                         "stream); the step's wall time is what to read")
    args = ap.parse_args(argv)
    pkg = pkgload.load()
    if args.replicated:
        return replicated(args, pkg)
    n_items, err, batch, _ = bench.CONFIGS[args.config]
    m = pkg.Bloomfilter.optimal_m(n_items, err)
    k = pkg.Bloomfilter.optimal_k(n_items, m)
    dev = torch.device("cuda", 0)
    eng = pkg.distributed.HipEngine(m, k, args.shards, 0, 20, dev)
    f = eng.filter
    if not args.no_prefill:   # bench.py's partitioned prefill: 50 % random bits in every shard
        sh = pkg.distributed.device_bytes_view(f, (f.local_bits + 7) // 8)
        g = torch.Generator(device=dev)
        g.manual_seed(bench.SEED * 7919)
        sh.random_(0, 256, generator=g)
    batches = bench.make_batches(n_items, batch, 0, args.steps + 1, dev)
    torch.cuda.synchronize()

    P = args.shards
    cap = batch * k // P + batch * k // (8 * P) + 4096

    nh = eng.nh   # 2^32-bit sub-range windows per owner (1 when the shard fits 2^32 bits)

    def received(send, counts):
        """Stand-in for the receive: every window's live entries, grouped by sub-range h
        (what the grouped send/recv delivers when every source routed this batch)."""
        c = counts.cpu().tolist()
        runs = []
        for h in range(nh):
            parts = [send[(s * nh + h) * cap: (s * nh + h) * cap + c[s * nh + h]] for s in range(P)]
            runs.append((h, torch.cat(parts)))
        return runs

    def step_windows(b):
        (ikb, iko), (qkb, qko) = b
        send, _, counts = eng.route_windows(ikb, iko, batch, cap, want_slot=False)
        for h, run in received(send, counts):
            eng.shard_insert_hi(run, h)
        send, slot, counts = eng.route_windows(qkb, qko, batch, cap)
        back = torch.empty(P * nh * cap, dtype=torch.uint8, device=dev)
        c = counts.cpu().tolist()
        for h, run in received(send, counts):
            bits = torch.empty(run.numel(), dtype=torch.uint8, device=dev)
            eng.shard_test_hi(run, h, bits)
            at = 0
            for s in range(P):
                w = s * nh + h
                back[w * cap: w * cap + c[w]] = bits[at: at + c[w]]
                at += c[w]
        return eng.combine_windows(back, slot, counts, cap, batch)

    def step_sf(b):
        (ikb, iko), (qkb, qko) = b
        A = 12288
        capsf = -(-min(batch * k, batch * k // P + batch * k // (8 * P) + 4096) // A) * A
        send, _, counts = eng.route_windows(ikb, iko, batch, capsf, want_slot=False)
        rmsg = torch.cat([counts.view(P, 1), torch.zeros(P, 1, dtype=torch.int64, device=dev)], 1).contiguous()
        eng.shard_insert_windows(send, capsf, P, rmsg, 0, 2, 0)
        send, slot, counts = eng.route_windows(qkb, qko, batch, capsf)
        rmsg = torch.cat([counts.view(P, 1), torch.zeros(P, 1, dtype=torch.int64, device=dev)], 1).contiguous()
        bits = torch.empty(P * capsf, dtype=torch.uint8, device=dev)
        eng.shard_test_windows(send, capsf, P, rmsg, 0, 2, 0, bits)
        cap8 = (capsf + 7) // 8
        seg = torch.tensor([[src * capsf, capsf, src * cap8] for src in range(P)], dtype=torch.int64).to(dev)
        packed = eng.pack_answers(bits, seg, capsf, P * cap8)
        return eng.combine_windows_packed(packed, slot, counts, capsf, batch)

    def step_chunks(b):
        (ikb, iko), (qkb, qko) = b
        A = 12288
        capsf = -(-min(batch * k, batch * k // P + batch * k // (8 * P) + 4096) // A) * A
        tiles, dbytes = eng.chunk_info(batch)
        perm = [o * nh + h for h in range(nh) for o in range(P)]   # receive slot h*P + src <- send window

        def deliver(send, dirb, counts):
            if nh == 1:
                recv, rdir = send, dirb
            else:   # the exchange's job (not a library kernel): windows into the receive layout
                recv = send.view(P * nh, capsf)[perm].reshape(-1)
                rdir = dirb.view(P * nh, dbytes)[perm].reshape(-1)
            rmsg = torch.cat([counts.view(P, nh), torch.zeros(P, 1, dtype=torch.int64, device=dev)], 1).contiguous()
            return recv, rdir, rmsg

        if args.overlap:   # this step's insert batch was routed during the previous step, on side
            torch.cuda.current_stream(dev).wait_event(pre["ev"])
            send, counts, dirb = pre["send"], pre["counts"], pre["dirb"]
        elif args.hash_split:   # SHA-1 in its own full-occupancy pass, then the route from the words
            send, _, counts, dirb = eng.route_chunks(eng.hash_keys(ikb, iko, batch, digs["ins"]), None, batch, capsf,
                                                     tiles, dbytes, want_slot=False)
        else:
            send, _, counts, dirb = eng.route_chunks(ikb, iko, batch, capsf, tiles, dbytes, want_slot=False)
        recv, rdir, rmsg = deliver(send, dirb, counts)
        fused = not (args.separate or args.dig or args.packed_bytes or args.overlap)
        if fused:   # the owner's insert and include? in one pass (bf_shard_insert_test_chunks_packed_dev)
            ins_recv = (recv, rdir, rmsg)
        else:
            eng.shard_insert_chunks(recv, capsf, P, rdir, dbytes, tiles, rmsg, nh + 1)
        if args.overlap:   # the next step's insert route, beside this step's owner kernels
            nb = nxt_batch[0]
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):   # a second handle: one handle orders its calls across streams
                s_, _, c_, d_ = router.route_chunks(nb[0][0], nb[0][1], batch, capsf, tiles, dbytes, want_slot=False)
                ev = torch.cuda.Event()
                ev.record(side)
            pre.update(send=s_, counts=c_, dirb=d_, ev=ev)
        if args.dig or args.fused_dig:   # this step's include? batch was hashed by the previous step's owner pass
            send, slot, counts, dirb = eng.route_chunks(digs["cur"], None, batch, capsf, tiles, dbytes)
        elif args.hash_split:
            send, slot, counts, dirb = eng.route_chunks(eng.hash_keys(qkb, qko, batch, digs["inc"]), None, batch,
                                                        capsf, tiles, dbytes)
        else:
            send, slot, counts, dirb = eng.route_chunks(qkb, qko, batch, capsf, tiles, dbytes)
        recv, rdir, rmsg = deliver(send, dirb, counts)
        if fused:
            nxt = None
            if args.fused_dig:   # ... and this pass hashes the next step's include? batch
                nq = nxt_batch[0][1]
                nxt = (nq[0], nq[1], batch, digs["spare"])
            packed = eng.shard_insert_test_chunks_packed(*ins_recv, recv, rdir, rmsg, capsf, P, dbytes, tiles, nh + 1,
                                                         nxt=nxt)
            if args.fused_dig:
                digs["spare"], digs["cur"] = digs["cur"], digs["spare"]
            return eng.combine_chunks_packed(packed, slot, capsf, dirb, dbytes, tiles, counts, batch)
        if not args.dig and not args.packed_bytes:   # the owner test writes the packed answers itself
            packed = eng.shard_test_chunks_packed(recv, capsf, P, rdir, dbytes, tiles, rmsg, nh + 1)
            return eng.combine_chunks_packed(packed, slot, capsf, dirb, dbytes, tiles, counts, batch)
        bits = torch.empty(nh * P * capsf, dtype=torch.uint8, device=dev)
        nxt = None
        if args.dig:   # ... and this one hashes the next step's
            nq = nxt_batch[0][1]
            nd = digs["spare"]
            nxt = (nq[0], nq[1], batch, nd)
            if args.dig_side:   # on a second stream, beside the test
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    hasher.hash_many_dev(nq[0].data_ptr(), nq[1].data_ptr(), batch, nd.data_ptr(),
                                         stream=side.cuda_stream)
                    hev = torch.cuda.Event()
                    hev.record(side)
                nxt = None
        eng.shard_test_chunks(recv, capsf, P, rdir, dbytes, tiles, rmsg, nh + 1, bits, nxt=nxt)
        if args.dig:
            if args.dig_side:
                torch.cuda.current_stream(dev).wait_event(hev)
            digs["spare"], digs["cur"] = digs["cur"], nd
        cap8 = (capsf + 7) // 8
        seg = torch.tensor([[(h * P + src) * capsf, capsf, (src * nh + h) * cap8] for src in range(P)
                            for h in range(nh)], dtype=torch.int64).to(dev)
        packed = eng.pack_answers(bits, seg, capsf, P * nh * cap8)
        return eng.combine_chunks_packed(packed, slot, capsf, dirb, dbytes, tiles, counts, batch)

    side = torch.cuda.Stream(dev)
    router = pkg.distributed.HipEngine(m, k, args.shards, 0, 20, dev) if args.overlap else None
    pre = {}
    nxt_batch = [None]
    digs = {}
    hasher = pkg.Filter(1 << 20, k, device=0) if args.dig_side else None   # hash_many needs a handle
    if args.hash_split:
        digs["ins"] = torch.empty((batch, 4), dtype=torch.int32, device=dev)
        digs["inc"] = torch.empty((batch, 4), dtype=torch.int32, device=dev)
    if args.dig or args.fused_dig:   # batch 0's include? words before the first step (the pipeline's fill)
        digs["cur"] = eng.hash_keys(batches[0][1][0], batches[0][1][1], batch)
        digs["spare"] = torch.empty_like(digs["cur"])

    def step(b):
        if args.chunks:
            return step_chunks(b)
        if args.sync_free:
            assert nh == 1
            return step_sf(b)
        if args.windows:
            return step_windows(b)
        (ikb, iko), (qkb, qko) = b
        send, _, _ = eng.route(ikb, iko, batch, want_slot=False)
        eng.shard_insert(send)
        send, slot, _ = eng.route(qkb, qko, batch)
        bits = eng.shard_test(send)
        return eng.combine(bits, slot, batch)

    if args.overlap:   # batch 0's insert route before the first step (the pipeline's fill)
        tiles0, dbytes0 = eng.chunk_info(batch)
        A = 12288
        cap0 = -(-min(batch * k, batch * k // P + batch * k // (8 * P) + 4096) // A) * A
        s_, _, c_, d_ = eng.route_chunks(batches[0][0][0], batches[0][0][1], batch, cap0, tiles0, dbytes0,
                                         want_slot=False)
        ev = torch.cuda.Event()
        ev.record()
        pre.update(send=s_, counts=c_, dirb=d_, ev=ev)
    nxt_batch[0] = batches[1]
    step(batches[0])
    torch.cuda.synchronize()
    f.profile(True)
    f.profile_read(reset=True)
    t0 = time.perf_counter()
    for i, b in enumerate(batches[1:], start=1):
        nxt_batch[0] = batches[(i + 1) % len(batches)]
        step(b)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    prof = f.profile_read(reset=True)
    out = {"config": args.config, "shards": args.shards, "m": m, "k": k, "batch": batch,
           "prefill": None if args.no_prefill else "50% random bits",
           "shard_bytes": f.device_bytes, "route32": bool(eng.offset_dtype == torch.int32),
           "hash_split": bool(args.chunks and args.hash_split),
           "route": "chunked windows" if args.chunks else
                    ("sync-free windows" if args.sync_free else ("windows" if args.windows else "contiguous")),
           "ms_per_step_compute": wall * 1e3,
           "kernels_ms_per_step": {name: ms / args.steps for name, (ms, _) in prof.items()},
           "kernels_ms_sum": sum(ms for ms, _ in prof.values()) / args.steps,
           "note": "per-rank compute = kernels_ms_sum; ms_per_step_compute also holds the stand-in receive "
                   "copies (--windows; --chunks with nh > 1: the windows permuted into the receive layout), "
                   "which are the exchange's job in a real run"}
    for e in (eng, router):
        if e is not None:
            e.close()
    if hasher is not None:
        hasher.close()
    return out


def replicated(args, pkg):
    """Per-replica compute of the replicated step at world size R, on one GPU: every rank's
    batch i (R x batch keys) goes in as one insert, then this rank's include? of batch i.
    The all-gather itself is not in these numbers (it runs beside the previous step)."""
    R = args.replicated
    n_items, err, batch, _ = bench.CONFIGS[args.config]
    m = pkg.Bloomfilter.optimal_m(n_items, err)
    k = pkg.Bloomfilter.optimal_k(n_items, m)
    dev = torch.device("cuda", 0)
    f = pkg.Filter(m, k, device=0)
    bench.prefill_random(f, m, k, 0, host_copy=False)
    steps = []
    for st in range(args.steps + 1):   # each step: R ranks' insert batches + one include? batch
        per = [bench.make_batches(n_items, batch, r + 1000 * st, 1, dev)[0] for r in range(R)]
        kbs, offs, base = [], [], 0
        for (ikb, iko), _ in per:
            nb = int(iko[-1].item())
            kbs.append(ikb[:nb])
            offs.append(iko[:-1] + base)
            base += nb
        mkb = torch.cat(kbs + [torch.zeros(16, dtype=torch.uint8, device=dev)])
        mko = torch.cat(offs + [torch.tensor([base], dtype=torch.int64, device=dev)])
        dg = None
        if args.gathered == "digests":   # the words every rank's batch arrives as (hashed by its rank)
            dg = torch.empty((R * batch, 4), dtype=torch.int32, device=dev)
            f.hash_many_dev(mkb.data_ptr(), mko.data_ptr(), R * batch, dg.data_ptr())
        elif args.gathered == "sets":   # what the all-gather delivers: every rank's set buffer (rank 0 = own,
            # re-encoded inside the timed step)
            cap = f.region_sets_capacity(batch)
            dg = torch.empty(R * (cap // 4), dtype=torch.int32, device=dev)
            for r, ((ikb, iko), _) in enumerate(per):
                f.encode_region_sets_dev(ikb.data_ptr(), iko.data_ptr(), batch, dg[r * (cap // 4):].data_ptr(), cap)
            torch.cuda.synchronize()
            mkb, mko = per[0][0]   # own batch's keys
        steps.append((mkb, mko, per[0][1], dg))
    nm = R * batch
    out = torch.empty(batch, dtype=torch.uint8, device=dev)
    own = torch.empty((batch, 4), dtype=torch.int32, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream

    cap_sets = f.region_sets_capacity(batch) if args.gathered == "sets" else 0

    def step(s_, nxt_=None):
        mkb, mko, (qkb, qko), dg = s_
        if args.gathered == "sets" and args.fused_hash:   # own words from the previous include? kernel
            f.encode_region_sets_digests_dev(own.data_ptr(), batch, dg.data_ptr(), cap_sets, stream=sp)
            f.insert_region_sets_dev(dg.data_ptr(), cap_sets, R, R * batch * k, d_any_new=flag.data_ptr(), stream=sp)
            nkb, nko = nxt_[0], nxt_[1]   # the next step's own batch, hashed here
            f.include_hash_dev(qkb.data_ptr(), qko.data_ptr(), batch, out.data_ptr(), nkb.data_ptr(), nko.data_ptr(),
                               batch, own.data_ptr(), stream=sp)
            return
        if args.gathered == "sets":   # own batch sorted + encoded (into rank 0's slot), then all R sets in
            f.encode_region_sets_dev(mkb.data_ptr(), mko.data_ptr(), batch, dg.data_ptr(), cap_sets, stream=sp)
            f.insert_region_sets_dev(dg.data_ptr(), cap_sets, R, R * batch * k, d_any_new=flag.data_ptr(), stream=sp)
        elif args.gathered == "digests":   # this rank hashes its own batch; all R batches go in from words
            f.hash_many_dev(mkb.data_ptr(), mko.data_ptr(), batch, own.data_ptr(), stream=sp)
            f.insert_digests_dev(dg.data_ptr(), nm, d_any_new=flag.data_ptr(), stream=sp)
        else:
            f.insert_many_dev(mkb.data_ptr(), mko.data_ptr(), nm, d_any_new=flag.data_ptr(), stream=sp)
        f.include_many_dev(qkb.data_ptr(), qko.data_ptr(), batch, out.data_ptr(), stream=sp)

    ovl = args.overlap_encode
    if args.fused_encode:
        assert args.gathered == "sets" and args.fused_hash and not ovl
        # one kernel per step for this step's sets (apply) and the next batch's own set (encode,
        # bf_insert_encode_region_sets_dev); the include? hashes the batch after next
        owns = [own, torch.empty_like(own)]

        def step_fe(j):
            s_, n1, n2 = steps[j % len(steps)], steps[(j + 1) % len(steps)], steps[(j + 2) % len(steps)]
            _, _, (qkb, qko), dg = s_
            f.insert_encode_region_sets_dev(dg.data_ptr(), cap_sets, R, R * batch * k, owns[(j + 1) % 2].data_ptr(),
                                            batch, n1[3].data_ptr(), cap_sets, d_any_new=flag.data_ptr(), stream=sp)
            f.include_hash_dev(qkb.data_ptr(), qko.data_ptr(), batch, out.data_ptr(), n2[0].data_ptr(),
                               n2[1].data_ptr(), batch, owns[j % 2].data_ptr(), stream=sp)

        # the pipeline's fill: batch 0's words and set, batch 1's words
        f.hash_many_dev(steps[0][0].data_ptr(), steps[0][1].data_ptr(), batch, owns[0].data_ptr(), stream=sp)
        f.encode_region_sets_digests_dev(owns[0].data_ptr(), batch, steps[0][3].data_ptr(), cap_sets, stream=sp)
        f.hash_many_dev(steps[1][0].data_ptr(), steps[1][1].data_ptr(), batch, owns[1].data_ptr(), stream=sp)
        step_fe(0)
        torch.cuda.synchronize()
        f.profile(True)
        f.profile_read(reset=True)
        t0 = time.perf_counter()
        for j in range(1, args.steps + 1):
            step_fe(j)
        torch.cuda.synchronize()
    elif ovl:
        assert args.gathered == "sets" and args.fused_hash
        # the encoder: a bitset-less handle (BF_FLAG_ENCODER) with its own scratch, so its calls are
        # not ordered behind the main handle's (ReplicatedFilter's side_encode)
        enc = pkg.Filter(m, k, device=0, flags=pkg._lib.BF_FLAG_ENCODER)
        side = torch.cuda.Stream(dev, priority=-1 if args.side_priority else 0)
        owns = [own, torch.empty_like(own)]
        main_s = torch.cuda.current_stream(dev)
        if args.main_priority:   # the step's own kernels on a high-priority queue, the encode beside them
            main_s = torch.cuda.Stream(dev, priority=-1)
            main_s.wait_stream(torch.cuda.current_stream(dev))
            sp = main_s.cuda_stream

        def step_ovl(j):
            s_, n1, n2 = steps[j % len(steps)], steps[(j + 1) % len(steps)], steps[(j + 2) % len(steps)]
            # side: the next step's own sets, from the words the previous include? hashed
            side.wait_stream(main_s)
            if ovl == "include":   # ... once this step's sets are in
                main_s.wait_event(pend[0])
                _, _, (qkb, qko), dg = s_
                f.insert_region_sets_dev(dg.data_ptr(), cap_sets, R, R * batch * k, d_any_new=flag.data_ptr(),
                                         stream=sp)
                side.wait_stream(main_s)
            enc.encode_region_sets_digests_dev(owns[(j + 1) % 2].data_ptr(), batch, n1[3].data_ptr(), cap_sets,
                                               stream=side.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(side)
            # main: this step's sets (encoded during the previous step) in, then the include?
            if ovl == "apply":
                main_s.wait_event(pend[0])
                _, _, (qkb, qko), dg = s_
                f.insert_region_sets_dev(dg.data_ptr(), cap_sets, R, R * batch * k, d_any_new=flag.data_ptr(),
                                         stream=sp)
            f.include_hash_dev(qkb.data_ptr(), qko.data_ptr(), batch, out.data_ptr(), n2[0].data_ptr(),
                               n2[1].data_ptr(), batch, owns[j % 2].data_ptr(), stream=sp)
            pend[0] = ev

        pend = [None]
        # the pipeline's fill: batch 0's words and sets, batch 1's words
        f.hash_many_dev(steps[0][0].data_ptr(), steps[0][1].data_ptr(), batch, owns[0].data_ptr(), stream=sp)
        f.encode_region_sets_digests_dev(owns[0].data_ptr(), batch, steps[0][3].data_ptr(), cap_sets, stream=sp)
        f.hash_many_dev(steps[1][0].data_ptr(), steps[1][1].data_ptr(), batch, owns[1].data_ptr(), stream=sp)
        pend[0] = torch.cuda.Event()
        pend[0].record(main_s)
        step_ovl(0)
        torch.cuda.synchronize()
        f.profile(True)
        f.profile_read(reset=True)
        enc.profile(True)
        enc.profile_read(reset=True)
        t0 = time.perf_counter()
        for j in range(1, args.steps + 1):
            step_ovl(j)
        torch.cuda.synchronize()
    else:
        if args.fused_hash:   # the pipeline's fill: the first step's own words
            f.hash_many_dev(steps[0][0].data_ptr(), steps[0][1].data_ptr(), batch, own.data_ptr(), stream=sp)
        step(steps[0], steps[1 % len(steps)])
        torch.cuda.synchronize()
        f.profile(True)
        f.profile_read(reset=True)
        t0 = time.perf_counter()
        for j, s_ in enumerate(steps[1:], start=1):
            step(s_, steps[(j + 1) % len(steps)])
        torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    prof = f.profile_read(reset=True)
    if ovl:
        for name, (ms, n) in enc.profile_read(reset=True).items():
            prof["side:" + name] = (ms, n)
        enc.close()
    if os.environ.get("BFHIP_SETS_STOP", "0") == "0":   # (the encode stop-point A/B writes no sets)
        assert out.cpu().numpy()[: batch // 2].all(), "false negative"
    res = {"config": args.config, "layout": "replicated", "world": R, "gathered": args.gathered,
           "fused_hash": bool(args.fused_hash), "overlap_encode": ovl or None,
           "main_priority": bool(ovl and args.main_priority), "side_priority": bool(ovl and args.side_priority),
           "fused_encode": bool(args.fused_encode),
           "m": m, "k": k,
           "batch": batch, "merged_insert_keys": nm, "bitset_bytes": f.device_bytes,
           "gathered_bytes_per_rank": (cap_sets if args.gathered == "sets" else
                                       batch * 16 if args.gathered == "digests" else None),
           "sets_used_bytes_per_rank": int(steps[-1][3][3].item()) * 4 if args.gathered == "sets" else None,
           "ms_per_step_compute": wall * 1e3,
           "kernels_ms_per_step": {name: ms / args.steps for name, (ms, _) in prof.items()},
           "kernels_ms_sum": sum(ms for ms, _ in prof.values()) / args.steps,
           "keys_per_s_per_rank": 2 * batch / wall,
           "note": "one replica's kernels per step at world size R; the key all-gather runs beside the "
                   "previous step and is not included"}
    f.close()
    return res


if __name__ == "__main__":
    main()
