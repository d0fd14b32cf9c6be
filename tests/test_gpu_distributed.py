"""Partitioned-filter primitives on the GPU (route / shard insert / shard test /
combine through the C ABI), with P shards simulated in one process on one
MI355X, plus the torch.distributed layer at world size 1 over RCCL.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def dev_batch(pkg, torch, keys):
    buf, offs = pkg.keys.pack(keys)
    kb = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).cuda()
    ko = torch.from_numpy(offs.view(np.int64)).cuda()
    return kb, ko, len(offs) - 1, buf, offs


# both owner forms (direct / binned) on the small and north-star filters; the 10B and 200B
# filters (the slow cases) once each, on the form their owners take
@pytest.mark.parametrize("m,k,P,b,binned", [
    (95851, 6, 3, 10, "0"), (95851, 6, 3, 10, "1"),
    (9585058377, 6, 8, 20, "0"), (9585058377, 6, 8, 20, "1"),
    (191701167547, 13, 4, 20, "1"),
    (3834023350947, 13, 8, 20, "0"),   # 200B@0.01 % over 8 GPUs (BASELINE configs[4])
])
def test_simulated_partition(pkg, oracle, monkeypatch, m, k, P, b, binned):
    """binned=1 forces the owner-side binned insert (offsets front pass + region apply) and
    binned shard test, and takes the wave-aggregated owner ranks in the route; 0 the direct
    kernels and LDS atomics."""
    import torch
    monkeypatch.setenv("BFHIP_INSERT_BINNED", binned)
    monkeypatch.setenv("BFHIP_SHARD_TEST_BINNED", binned)
    monkeypatch.setenv("BFHIP_ROUTE_AGG", "16" if binned == "1" else "0")
    D = pkg.distributed
    dev = torch.device("cuda", 0)
    shards = [D.HipEngine(m, k, P, s, b, dev) for s in range(P)]
    rng = np.random.default_rng(9)
    per_rank = [["p%d-%d" % (r, int(v)) for v in rng.integers(0, 10**9, 4000)] for r in range(P)]
    routed = []
    for r in range(P):
        kb, ko, n, buf, offs = dev_batch(pkg, torch, per_rank[r])
        send, slot, counts = shards[r].route(kb, ko, n)
        torch.cuda.synchronize()
        # route invariants vs the oracle: every probe lands in its owner's segment at the right local offset
        idx = oracle.indexes_many(buf, offs, m, k).reshape(-1)
        owner, local = D.block_owner_local(idx, P, b)
        c = counts.cpu().numpy()
        assert c.tolist() == np.bincount(owner, minlength=P).tolist()
        s_np = send.cpu().numpy()   # int32 when the shards fit 2^32 bits (BF_FLAG_ROUTE32)
        s_np = s_np.view(np.uint32).astype(np.uint64) if s_np.dtype == np.int32 else s_np.view(np.uint64)
        assert (send.dtype == torch.int32) == shards[r].filter.route32
        sl = slot.cpu().numpy().astype(np.int64)   # key index of every send entry
        assert np.bincount(sl, minlength=n).tolist() == [k] * n
        displ = np.concatenate([[0], np.cumsum(c)[:-1]])
        key_of = np.arange(n * k) // k
        for s in range(P):   # owner s's segment holds exactly its (key, local) pairs
            seg = slice(int(displ[s]), int(displ[s] + c[s]))
            got = sorted(zip(sl[seg].tolist(), s_np[seg].tolist()))
            want = sorted(zip(key_of[owner == s].tolist(), local[owner == s].tolist()))
            assert got == want
        routed.append((send, slot, c, displ, n))
    # exchange: owner s receives every rank's segment s
    for s in range(P):
        recv = torch.cat([send[int(d[s]):int(d[s] + c[s])] for send, _, c, d, _ in routed])
        shards[s].shard_insert(recv)
    torch.cuda.synchronize()
    ib, io = pkg.keys.pack([x for r in range(P) for x in per_rank[r]])
    bits = oracle.new_bitset(m, k)
    oracle.insert_many(bits, m, k, ib, io)
    want_str = oracle.redis_string(bits)
    got_str = D.interleave_shards([e.shard_export() for e in shards], shards[0].filter.reach_bits, b)
    assert got_str == want_str
    # include?: members of every rank + fresh keys, answered via owners and combined
    probe = per_rank[0][:2000] + per_rank[P - 1][:2000] + ["fresh%d" % i for i in range(4000)]
    kb, ko, n, pb, po = dev_batch(pkg, torch, probe)
    send, slot, counts = shards[1 % P].route(kb, ko, n)
    c = counts.cpu().numpy()
    d = np.concatenate([[0], np.cumsum(c)[:-1]])
    back = torch.empty(n * k, dtype=torch.uint8, device=dev)
    for s in range(P):
        seg = send[int(d[s]):int(d[s] + c[s])]
        back[int(d[s]):int(d[s] + c[s])] = shards[s].shard_test(seg)
    got = shards[1 % P].combine(back, slot, n).cpu().numpy()
    want = oracle.include_many(bits, m, k, pb, po)
    np.testing.assert_array_equal(got, want)
    # every owner's answer byte is the bit at that probe's global offset
    s_np = send.cpu().numpy()
    s_np = s_np.view(np.uint32).astype(np.uint64) if s_np.dtype == np.int32 else s_np.view(np.uint64)
    owner_of = np.repeat(np.arange(P), c)
    lblk, low = s_np >> np.uint64(b), s_np & np.uint64((1 << b) - 1)
    glob = ((lblk * np.uint64(P) + owner_of.astype(np.uint64)) << np.uint64(b)) | low
    want_bits = (bits.view(np.uint8)[(glob >> np.uint64(3)).astype(np.int64)] >> (7 - (glob & np.uint64(7))).astype(np.uint8)) & 1
    np.testing.assert_array_equal(back.cpu().numpy(), want_bits)
    for e in shards:
        e.close()


@pytest.mark.parametrize("m,k,P,b", [(95851, 6, 3, 10), (9585058377, 6, 8, 20), (191701167547, 13, 4, 20),
                                     (9585058377, 6, 2, 20),
                                     (3834023350947, 13, 8, 20)])   # 200B at P = 8: nh = 2
def test_route_windows(pkg, oracle, m, k, P, b):
    """bf_route_windows_dev: window w = s*nh + hi holds exactly owner s's (key, local offset)
    pairs with local >> 32 == hi, as uint32 (the multiset bf_route_dev puts in segment s, split
    by sub-range); the owner's hi ops see (hi << 32) | entry; bf_combine_windows_dev over the
    window layout equals the AND; a window smaller than its probes shows in the counts.
    (9585058377, 6, 2) and the 10B cases: shards past 2^32 bits, so nh > 1."""
    import torch
    D = pkg.distributed
    dev = torch.device("cuda", 0)
    e = D.HipEngine(m, k, P, 0, b, dev)
    nh = e.nh
    want_nh = max(1, -(-D.shard_local_bits(min(m, k * 0xFFFFFFFF + 1), P, 0, b) // (1 << 32)))
    assert nh == want_nh
    if m == 3834023350947:
        assert nh == 2
    nwin = P * nh
    rng = np.random.default_rng(17)
    keys = ["w%d" % int(v) for v in rng.integers(0, 10**12, 30000)]
    kb, ko, n, buf, offs = dev_batch(pkg, torch, keys)
    idx = oracle.indexes_many(buf, offs, m, k).reshape(-1)
    owner, local = D.block_owner_local(idx, P, b)
    win = owner.astype(np.int64) * nh + (local >> np.uint64(32)).astype(np.int64)
    want_c = np.bincount(win, minlength=nwin)
    key_of = np.arange(n * k) // k
    cap = int(want_c.max()) + 37
    send, slot, counts = e.route_windows(kb, ko, n, cap)
    torch.cuda.synchronize()
    assert send.dtype == torch.int32
    assert counts.cpu().numpy().tolist() == want_c.tolist()
    s_np = send.cpu().numpy().view(np.uint32).astype(np.uint64)
    sl = slot.cpu().numpy().astype(np.int64)
    for w in range(nwin):
        ws = slice(w * cap, w * cap + int(want_c[w]))
        got = sorted(zip(sl[ws].tolist(), (s_np[ws] | np.uint64((w % nh) << 32)).tolist()))
        assert got == sorted(zip(key_of[win == w].tolist(), local[win == w].tolist()))
    # owner-side hi ops: shard 0 inserts its windows, then answers every probe of them
    ins = [(h, send[h * cap: h * cap + int(want_c[h])]) for h in range(nh)]
    for h, run in ins:
        e.shard_insert_hi(run, h)
    for h, run in ins:
        bits_h = torch.empty(run.numel(), dtype=torch.uint8, device=dev)
        e.shard_test_hi(run, h, bits_h)
        assert bool(bits_h.all())
    shard = e.shard_export()
    lo = local[owner == 0]
    want_shard = np.zeros_like(shard)
    np.bitwise_or.at(want_shard, (lo >> np.uint64(3)).astype(np.int64), (np.uint64(0x80) >> (lo & np.uint64(7))).astype(np.uint8))
    np.testing.assert_array_equal(shard, want_shard)
    # combine over windows: answer bytes from a known bitset
    bits = oracle.new_bitset(m, k)
    ib, io = pkg.keys.pack(keys[: n // 2])
    oracle.insert_many(bits, m, k, ib, io)
    ans = np.zeros(nwin * cap, np.uint8)
    for w in range(nwin):
        s_, h = divmod(w, nh)
        lw = s_np[w * cap: w * cap + int(want_c[w])] | np.uint64(h << 32)
        blk, low = lw >> np.uint64(b), lw & np.uint64((1 << b) - 1)
        glob = ((blk * np.uint64(P) + np.uint64(s_)) << np.uint64(b)) | low
        ans[w * cap: w * cap + int(want_c[w])] = \
            (bits.view(np.uint8)[(glob >> np.uint64(3)).astype(np.int64)] >> (7 - (glob & np.uint64(7))).astype(np.uint8)) & 1
    got = e.combine_windows(torch.from_numpy(ans).to(dev), slot, counts, cap, n).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.include_many(bits, m, k, buf, offs))
    assert got[: n // 2].all()
    # too-small windows: the counts still report every window's full total
    small = max(1, int(want_c[want_c > 0].min()) // 2)
    _, _, c2 = e.route_windows(kb, ko, n, small, want_slot=False)
    assert c2.cpu().numpy().tolist() == want_c.tolist()
    # an empty batch zeroes the counts
    _, _, c3 = e.route_windows(kb, ko, 0, 16)
    assert c3.cpu().numpy().tolist() == [0] * nwin
    e.close()


# every owner form on the small and north-star filters; the 10B x 4 and 200B x 8 filters (the
# slow cases) on one form each: the L2 sweep, and the sorted test their owners take
@pytest.mark.parametrize("m,k,P,b,owner", [
    *[(m_, k_, P_, b_, o) for (m_, k_, P_, b_) in [(95851, 6, 3, 10), (9585058377, 6, 8, 20), (9585058377, 6, 2, 20),
                                                   (9585058377, 6, 1, 20)]
      for o in ("direct", "sorted", "l2")],
    (191701167547, 13, 4, 20, "l2"),
    (3834023350947, 13, 8, 20, "sorted"),   # 200B x8: nh = 2
])
def test_chunked_windows(pkg, oracle, monkeypatch, m, k, P, b, owner):
    """bf_route_chunks_dev + the owner ops over chunked windows + bf_combine_chunks_packed_dev,
    with P shards simulated on one GPU and the exchange done by copies: every window holds
    exactly its owner's (key, local offset) pairs, the directories partition each window into
    one run per route tile, the owners' shards rebuild the oracle's Redis string and the
    requesters' answers equal the oracle's include? (odd ranks route their include? batch from
    SHA-1 words; every owner test also hashes a side batch, whose words equal hash_many's).
    owner: "direct" = the direct kernels over
    the same windows; "sorted" = the binned pass straight off the chunks (bin_mid, then the
    region apply / test); "l2" = the binned insert and the superbin-major L2-local test."""
    import torch
    binned = "0" if owner == "direct" else "1"
    monkeypatch.setenv("BFHIP_INSERT_BINNED", binned)
    monkeypatch.setenv("BFHIP_SHARD_TEST_BINNED", binned)
    monkeypatch.setenv("BFHIP_CHUNK_TEST_L2", "1" if owner == "l2" else "0")
    D = pkg.distributed
    dev = torch.device("cuda", 0)
    shards = [D.HipEngine(m, k, P, s, b, dev) for s in range(P)]
    nh = shards[0].nh
    nwin = P * nh
    n = 6000
    geo = shards[0].chunk_info(n)
    assert geo is not None and all(e.chunk_info(n) == geo for e in shards)
    tiles, dbytes = geo
    S = shards[0].filter.route_chunk_info(n)[2]
    rank_off = 4 * tiles + 2 * (S + 1) * tiles          # start[tiles], tab[(S + 1) * tiles], then rank[tiles]
    claim_off = -(-(rank_off + 2 * tiles) // 8) * 8    # ... and the 8-byte claim counter
    assert dbytes == -(-(claim_off + 8) // 16) * 16
    tile_keys = 2048 if k <= 6 else 1024
    assert tiles == -(-n // tile_keys)
    A = 12288
    cap = -(-min(n * k, n * k // P + n * k // (8 * P) + 4096) // A) * A
    rng = np.random.default_rng(23)
    per_rank = [["c%d-%d" % (r, int(v)) for v in rng.integers(0, 10**12, n)] for r in range(P)]

    def route_all(batches, want_slot, dig=False):
        """dig: odd ranks route from their keys' SHA-1 words (bf_route_chunks_digests_dev)."""
        out = []
        for r in range(P):
            kb, ko, nn, buf, offs = dev_batch(pkg, torch, batches[r])
            if dig and r % 2:
                out.append(shards[r].route_chunks(shards[r].hash_keys(kb, ko, nn), None, nn, cap, tiles, dbytes,
                                                  want_slot=want_slot) + (buf, offs))
            else:
                out.append(shards[r].route_chunks(kb, ko, nn, cap, tiles, dbytes, want_slot=want_slot) + (buf, offs))
        torch.cuda.synchronize()
        return out

    def check_route(send, slot, counts, dirb, buf, offs):
        idx = oracle.indexes_many(buf, offs, m, k).reshape(-1)
        owner, local = D.block_owner_local(idx, P, b)
        win = owner.astype(np.int64) * nh + (local >> np.uint64(32)).astype(np.int64)
        want_c = np.bincount(win, minlength=nwin)
        c = counts.cpu().numpy()
        assert c.tolist() == want_c.tolist()
        s_np = send.cpu().numpy().view(np.uint32).astype(np.uint64)
        sl = slot.cpu().numpy().view(np.uint16).astype(np.int64)
        d = dirb.cpu().numpy()
        key_of = np.arange(len(idx)) // k
        for w in range(nwin):
            dw = d[w * dbytes:(w + 1) * dbytes]
            start = dw[: 4 * tiles].view(np.uint32).astype(np.int64)
            tab = dw[4 * tiles: 4 * tiles + 2 * (S + 1) * tiles].view(np.uint16).reshape(S + 1, tiles)
            length = tab[S].astype(np.int64)
            assert (np.diff(tab.astype(np.int64), axis=0) >= 0).all()   # superbin runs in order
            # the chunks tile [0, count) of the window, one per route tile, runs monotone inside
            live = length > 0
            spans = sorted(zip(start[live].tolist(), (start[live] + length[live]).tolist()))
            at = 0
            for a, e in spans:
                assert a == at
                at = e
            assert at == int(want_c[w])
            # the rank table lists the claimed runs in window order (the owner's ranked chunks)
            rank = dw[rank_off: rank_off + 2 * tiles].view(np.uint16).astype(np.int64)
            nclaim = int(dw[claim_off: claim_off + 8].view(np.uint64)[0]) >> 40
            assert nclaim == int(live.sum()) and (rank[nclaim:] == 0).all()
            ranked = rank[:nclaim] - 1
            assert sorted(ranked.tolist()) == np.flatnonzero(live).tolist()
            assert (np.diff(start[ranked]) > 0).all()
            got, keys_w = [], []
            for t in np.flatnonzero(live):
                seg = slice(w * cap + int(start[t]), w * cap + int(start[t] + length[t]))
                got += (s_np[seg] | np.uint64((w % nh) << 32)).tolist()
                keys_w += (sl[seg] + t * tile_keys).tolist()
            assert sorted(zip(keys_w, got)) == sorted(zip(key_of[win == w].tolist(), local[win == w].tolist()))

    def deliver(routed, o):
        recv = torch.cat([routed[src][0][(o * nh + h) * cap:(o * nh + h + 1) * cap] for h in range(nh)
                          for src in range(P)])
        rdir = torch.cat([routed[src][3][(o * nh + h) * dbytes:(o * nh + h + 1) * dbytes] for h in range(nh)
                          for src in range(P)])
        rmsg = torch.zeros(P, nh + 1, dtype=torch.int64, device=dev)
        for src in range(P):
            rmsg[src, :nh] = routed[src][2][o * nh:(o + 1) * nh]
        return recv, rdir, rmsg

    ins = route_all(per_rank, want_slot=True)
    for r in range(P):
        check_route(*ins[r][:4], ins[r][4], ins[r][5])
    for o in range(P):
        recv, rdir, rmsg = deliver(ins, o)
        shards[o].shard_insert_chunks(recv, cap, P, rdir, dbytes, tiles, rmsg, nh + 1)
    torch.cuda.synchronize()
    ib, io = pkg.keys.pack([x for r in range(P) for x in per_rank[r]])
    bits = oracle.new_bitset(m, k)
    oracle.insert_many(bits, m, k, ib, io)
    got_str = D.interleave_shards([e.shard_export() for e in shards], shards[0].filter.reach_bits, b)
    assert got_str == oracle.redis_string(bits)
    # include?: members of two ranks + fresh keys per requester
    probes = [per_rank[r][: n // 3] + per_rank[(r + 1) % P][: n // 3] + ["fresh%d-%d" % (r, i) for i in range(n // 3)]
              for r in range(P)]
    qs = route_all(probes, want_slot=True, dig=True)
    for r in range(1, P, 2):
        check_route(*qs[r][:4], qs[r][4], qs[r][5])
    cap8 = (cap + 7) // 8
    answers, packed_by_owner = [], []
    for o in range(P):
        recv, rdir, rmsg = deliver(qs, o)
        out = torch.zeros(nh * P * cap, dtype=torch.uint8, device=dev)
        # the owner test also hashes a side batch (a requester's next include? batch)
        skb, sko, sn, _, _ = dev_batch(pkg, torch, per_rank[o][: 3001 + 97 * o])
        sdig = torch.full((sn, 4), -1, dtype=torch.int32, device=dev)
        shards[o].shard_test_chunks(recv, cap, P, rdir, dbytes, tiles, rmsg, nh + 1, out, nxt=(skb, sko, sn, sdig))
        torch.testing.assert_close(sdig, shards[o].hash_keys(skb, sko, sn), rtol=0, atol=0)
        answers.append(out)
        # the packed form (bf_shard_test_chunks_packed_dev: ordered chunks + unsort for "sorted",
        # bytes + pack for the others): every live entry's bit equals its answer byte
        pk = shards[o].shard_test_chunks_packed(recv, cap, P, rdir, dbytes, tiles, rmsg, nh + 1).cpu().numpy()
        ob = out.cpu().numpy()
        cnt = rmsg.cpu().numpy()
        for src in range(P):
            for h in range(nh):
                live = int(cnt[src, h])
                bits_w = np.unpackbits(pk[(src * nh + h) * cap8:(src * nh + h + 1) * cap8], bitorder="little")
                np.testing.assert_array_equal(bits_w[:live], ob[(h * P + src) * cap:(h * P + src) * cap + live])
        packed_by_owner.append(torch.from_numpy(pk).to(dev))
    for r in range(P):   # the requesters' answers from the packed owner tests
        back = torch.cat([packed_by_owner[o][(r * nh) * cap8:(r * nh + nh) * cap8] for o in range(P)])
        send, slot, counts, dirb, pb, po = qs[r]
        got = shards[r].combine_chunks_packed(back, slot, cap, dirb, dbytes, tiles, counts, len(probes[r]))
        np.testing.assert_array_equal(got.cpu().numpy(), oracle.include_many(bits, m, k, pb, po))
    # the step's owner work in one pass (bf_shard_insert_test_chunks_packed_dev) on fresh shards:
    # the inserts land as the separate insert's did and every answer sees them
    fresh = [D.HipEngine(m, k, P, s_, b, dev) for s_ in range(P)]
    packed_f = []
    for o in range(P):   # ... and the pass hashes a side batch (the requester's next include? batch)
        skb, sko, sn, _, _ = dev_batch(pkg, torch, per_rank[o][: 2999 + 61 * o])
        sdig = torch.full((sn, 4), -1, dtype=torch.int32, device=dev)
        packed_f.append(fresh[o].shard_insert_test_chunks_packed(*deliver(ins, o), *deliver(qs, o), cap, P, dbytes,
                                                                 tiles, nh + 1, nxt=(skb, sko, sn, sdig)))
        torch.testing.assert_close(sdig, fresh[o].hash_keys(skb, sko, sn), rtol=0, atol=0)
    torch.cuda.synchronize()
    assert D.interleave_shards([e.shard_export() for e in fresh], fresh[0].filter.reach_bits, b) == got_str
    for r in range(P):
        back = torch.cat([packed_f[o][(r * nh) * cap8:(r * nh + nh) * cap8] for o in range(P)])
        send, slot, counts, dirb, pb, po = qs[r]
        got = fresh[r].combine_chunks_packed(back, slot, cap, dirb, dbytes, tiles, counts, len(probes[r]))
        np.testing.assert_array_equal(got.cpu().numpy(), oracle.include_many(bits, m, k, pb, po))
    for e in fresh:
        e.close()
    for r in range(P):
        back = torch.zeros(nwin * cap8, dtype=torch.uint8, device=dev)
        for o in range(P):
            seg = torch.tensor([[(h * P + r) * cap, cap, (o * nh + h) * cap8] for h in range(nh)],
                               dtype=torch.int64).to(dev)
            packed = shards[o].pack_answers(answers[o], seg, cap, nwin * cap8)
            back[o * nh * cap8:(o + 1) * nh * cap8] = packed[o * nh * cap8:(o + 1) * nh * cap8]
        send, slot, counts, dirb, pb, po = qs[r]
        got = shards[r].combine_chunks_packed(back, slot, cap, dirb, dbytes, tiles, counts, len(probes[r]))
        np.testing.assert_array_equal(got.cpu().numpy(), oracle.include_many(bits, m, k, pb, po))
    for e in shards:
        e.close()


def test_pack_segments_and_packed_combine(pkg):
    """bf_pack_segments_dev at odd offsets and counts (LSB-first, ceil(count/8) bytes each),
    and bf_combine_windows_packed_dev equal to the byte-per-probe windowed combine."""
    import torch
    D = pkg.distributed
    dev = torch.device("cuda", 0)
    e = D.HipEngine(95851, 6, 3, 0, 10, dev)
    rng = np.random.default_rng(3)
    bits = rng.integers(0, 2, 100_003).astype(np.uint8)
    segs = [(0, 0), (0, 1), (5, 13), (100, 8), (1001, 40_000), (41_001, 59_002)]
    pk = [(c + 7) // 8 for _, c in segs]
    dst = np.concatenate([[0], np.cumsum(pk)[:-1]]).tolist()
    seg = torch.tensor([[o, c, d] for (o, c), d in zip(segs, dst)], dtype=torch.int64).to(dev)
    got = e.pack_answers(torch.from_numpy(bits).to(dev), seg, max(c for _, c in segs), sum(pk)).cpu().numpy()
    for (o, c), d, k_ in zip(segs, dst, pk):
        np.testing.assert_array_equal(got[d: d + k_], np.packbits(bits[o: o + c], bitorder="little"))
    # packed combine == byte combine over 4 windows
    cap, nwin, n = 1000, 4, 700
    counts = np.array([0, 999, 1000, 537], np.int64)
    slot = rng.integers(0, n, nwin * cap).astype(np.int32)
    ans = rng.integers(0, 2, nwin * cap).astype(np.uint8) | (rng.random(nwin * cap) < 0.9).astype(np.uint8)
    cap8 = (cap + 7) // 8
    packed = np.concatenate([np.packbits(ans[w * cap: (w + 1) * cap], bitorder="little")[:cap8] for w in range(nwin)])
    t = lambda a: torch.from_numpy(a).to(dev)
    ct = t(counts)
    e.P = nwin   # the combine takes the window count from counts
    want = e.combine_windows(t(ans), t(slot), ct, cap, n).cpu().numpy()
    got = e.combine_windows_packed(t(packed), t(slot), ct, cap, n).cpu().numpy()
    np.testing.assert_array_equal(got, want)
    assert (want == 0).any() and (want == 1).any()
    e.close()


@pytest.mark.parametrize("binned", ["0", "1"])
def test_owner_ops_drop_offsets_past_the_shard(pkg, monkeypatch, binned):
    """Owner-side insert / test over caller-supplied device offsets never touch memory past the
    handle's local bits: such an offset is dropped by the insert and answers 0 in the test, on
    the direct and the binned passes; a combine slot >= n is ignored.  The bad offsets lie in
    the bitset allocation's rounding slack, so the check sees a dropped offset apart from an
    honoured one without relying on a fault."""
    import torch
    monkeypatch.setenv("BFHIP_INSERT_BINNED", binned)
    monkeypatch.setenv("BFHIP_SHARD_TEST_BINNED", binned)
    D = pkg.distributed
    m = 95851
    f = pkg.Filter(m, 6, device=0)
    _, total = f.device_bits()   # allocation bytes, rounded up to 256
    assert total * 8 > m + 64
    view = D.device_bytes_view(f)
    rng = np.random.default_rng(5)
    good = rng.integers(0, m, 3000).astype(np.int64)
    bad = np.array([m, m + 1, m + 63, total * 8 - 1], np.int64)
    local = torch.from_numpy(np.concatenate([good, bad])).cuda()
    f.shard_insert_dev(local.data_ptr(), local.numel(), stream=0)
    torch.cuda.synchronize()
    want = np.zeros(total, np.uint8)
    np.bitwise_or.at(want, (good >> 3).astype(np.int64), (0x80 >> (good & 7)).astype(np.uint8))
    np.testing.assert_array_equal(view.cpu().numpy(), want)
    # every bit past m set by hand: a test of an offset there still answers 0
    view[m >> 3] |= (1 << (8 - (m & 7))) - 1
    view[(m >> 3) + 1:] = 0xFF
    out = torch.empty(local.numel(), dtype=torch.uint8, device="cuda")
    f.shard_test_dev(local.data_ptr(), local.numel(), out.data_ptr(), stream=0)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert o[: len(good)].all() and not o[len(good):].any()
    # combine (n keys x k probes): a 0 answer whose slot is past the n keys is ignored
    n = 10
    sl = (np.arange(n * 6) // 6).astype(np.int32)
    sl[7], sl[13] = n + 5, 2 * n
    b = np.ones(n * 6, np.uint8)
    b[[7, 13, 20]] = 0   # two stray slots, and one real 0 answer for key 20 // 6 = 3
    ans = torch.full((n + 64,), 7, dtype=torch.uint8, device="cuda")
    bits_t, slot_t = torch.from_numpy(b).cuda(), torch.from_numpy(sl).cuda()
    f.combine_dev(bits_t.data_ptr(), slot_t.data_ptr(), n, ans.data_ptr(), stream=0)
    torch.cuda.synchronize()
    a = ans.cpu().numpy()
    assert a[:n].tolist() == [1, 1, 1, 0, 1, 1, 1, 1, 1, 1] and (a[n:] == 7).all()
    f.close()


def _trace(torch, *a):
    """BF_TRACE=1 (with pytest -s): a synchronize + progress line after each step."""
    if os.environ.get("BF_TRACE"):
        torch.cuda.synchronize()
        print("[world1]", *a, flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("poison", [None, "zero-bit"])
def test_torch_distributed_world1(pkg, oracle, monkeypatch, poison):
    """PartitionedFilter and ReplicatedFilter over RCCL (world size 1) match a single filter.

    poison="zero-bit" (VERDICT r02 item 6): every exchange buffer is filled before it is
    written — routed entries with the offset of a bit the oracle leaves 0, answer bytes with
    0 — so a kernel that reads an entry past a window's live count (the r02 fault) sets that
    bit or turns a member false, deterministically, instead of depending on what the caching
    allocator hands back.  The forced-overflow cases below run under it."""
    import torch
    import torch.distributed as dist
    if poison:
        ob = oracle.new_bitset(9585058, 6)
        ib_, io_ = pkg.keys.pack(["k%d" % i for i in range(50_000)])
        oracle.insert_many(ob, 9585058, 6, ib_, io_)
        raw = np.unpackbits(ob.view(np.uint8))
        monkeypatch.setenv("BFHIP_POISON_WINDOWS", str(int(np.flatnonzero(raw == 0)[0])))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        D = pkg.distributed
        m, k = 9585058, 6
        keys = ["k%d" % i for i in range(50_000)]
        probe = keys[:20_000] + ["x%d" % i for i in range(20_000)]
        ib, io = pkg.keys.pack(keys)
        pb, po = pkg.keys.pack(probe)
        bits = oracle.new_bitset(m, k)
        oracle.insert_many(bits, m, k, ib, io)
        want = oracle.include_many(bits, m, k, pb, po).astype(bool)
        for cls, kw in ((D.PartitionedFilter, {"block_log2": 16}), (D.ReplicatedFilter, {}),
                        (D.ReplicatedFilter, {"insert_mode": "or"})):
            f = cls(m, k, **kw)
            f.insert_many(keys)
            _trace(torch, cls.__name__, kw, "insert")
            np.testing.assert_array_equal(f.include_many(probe), want)
            _trace(torch, "include")
            assert f.export_redis() == oracle.redis_string(bits)
            _trace(torch, "export")
            if cls is D.PartitionedFilter:   # per-rank SETRANGE of the rank's blocks
                r = pkg.FakeRedis()
                r.set("bf", b"stale")
                f.write_redis(r, "bf", chunk_bytes=1 << 14)
                assert r.get("bf") == oracle.redis_string(bits)
                _trace(torch, "write_redis")
            f.close()
        # the overlapped insert + include? step (async RCCL sends beside the kernels), through
        # the window route, the contiguous route, and the overflow fallback
        # sync-free (default) and synced exchanges, forced overflows of each (the sync-free one
        # replays the step through the synced path), bytes instead of bits on the way back
        for kw, cap in (({}, None), ({"windows": False}, None), ({"sync_free": False}, 5), ({}, "sf"),
                        ({"pack_answers": False}, None), ({"pack_answers": False, "sync_free": False}, None)):
            f = D.PartitionedFilter(m, k, block_log2=16, **kw)
            if cap == "sf":
                f._cap_sf = lambda n: f.WINDOW_ALIGN   # 12288 < 50k keys x 6 probes: every batch overflows
            elif cap is not None:
                f._cap = lambda n, c=cap: c
            assert f.sync_free == (kw.get("sync_free", True) and kw.get("windows", True))
            np.testing.assert_array_equal(f.insert_include(keys, probe), want)
            _trace(torch, "insert_include", kw, cap)
            assert f.export_redis() == oracle.redis_string(bits)
            assert f.window_overflows == (2 if cap == 5 else 0)
            assert f.replays == (1 if cap == "sf" else 0)
            f.close()
        # the sync-free insert and include? calls on their own
        f = D.PartitionedFilter(m, k, block_log2=16)
        f.insert_many(keys)
        np.testing.assert_array_equal(f.include_many(probe), want)
        f.close()
        # a shard past 2^32 bits (the north-star filter, 1.2 GB, in one shard): the window
        # route splits it into nh = 3 sub-range windows of uint32 entries
        m, k = 9585058377, 6
        bits = oracle.new_bitset(m, k)
        oracle.insert_many(bits, m, k, ib, io)
        want = oracle.include_many(bits, m, k, pb, po).astype(bool)
        for kw in ({}, {"windows": False}):
            f = D.PartitionedFilter(m, k, block_log2=20, **kw)
            assert f.engine.nh == 3
            np.testing.assert_array_equal(f.insert_include(keys, probe), want)
            _trace(torch, "1.2 GB insert_include", kw)
            shard = f.engine.shard_export()
            assert np.array_equal(shard[: len(bits.view(np.uint8))], bits.view(np.uint8)[: len(shard)])
            f.close()
    finally:
        dist.destroy_process_group()


def test_route32_needs_small_shards(pkg):
    with pytest.raises(pkg.ArgumentError, match="ROUTE32"):
        pkg.Filter(191701167547, 13, shard_count=2, shard_index=0, flags=pkg._lib.BF_FLAG_ROUTE32)
    f = pkg.Filter(9585058377, 6, shard_count=4, shard_index=1, flags=pkg._lib.BF_FLAG_ROUTE32)
    assert f.route32 and f.local_bits <= 1 << 32
    f.close()
