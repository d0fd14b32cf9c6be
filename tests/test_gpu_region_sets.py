"""Replicated inserts from region sets (include/bfhip.h: bf_region_sets_capacity,
bf_encode_region_sets_dev / _digests_dev, bf_insert_region_sets_dev) against the oracle.

* the encoding itself: every region's decoded set (tests/sets_codec.py, a host reader
  independent of the device decoder) equals the distinct offsets the oracle derives for the
  batch (ruby.rb:41-55), in Elias-Fano and bitmap form, at 2^19- and 2^18-bit regions;
* the insert: the sets of several batches ORed into a filter give the bitset inserting all of
  their keys gives (ruby.rb:57-63), on an empty and a prefilled filter, with any_new as the
  reference's !found (ruby.rb:61); a foreign buffer is skipped and flagged."""
import numpy as np
import pytest

import sets_codec

pytestmark = pytest.mark.gpu

SEED = 0x5EED + 404


def _dev(torch, buf, offs):
    kb = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).cuda()
    ko = torch.from_numpy(offs.view(np.int64)).cuda()
    return kb, ko


def _keys(pkg, rng, n, tag="s"):
    return pkg.keys.pack(["%s%d" % (tag, int(v)) for v in rng.integers(0, 10**12, size=n)])


def _encode(torch, f, buf, offs, digests=False, cap=None):
    n = len(offs) - 1
    cap = cap or f.region_sets_capacity(n)
    sets = torch.zeros(cap // 4, dtype=torch.int32, device="cuda")
    if n and digests:
        kb, ko = _dev(torch, buf, offs)
        dig = torch.empty((n, 4), dtype=torch.int32, device="cuda")
        f.hash_many_dev(kb.data_ptr(), ko.data_ptr(), n, dig.data_ptr(), stream=0)
        f.encode_region_sets_digests_dev(dig.data_ptr(), n, sets.data_ptr(), cap, stream=0)
    elif n:
        kb, ko = _dev(torch, buf, offs)
        f.encode_region_sets_dev(kb.data_ptr(), ko.data_ptr(), n, sets.data_ptr(), cap, stream=0)
    else:
        f.encode_region_sets_dev(0, 0, 0, sets.data_ptr(), cap, stream=0)
    torch.cuda.synchronize()
    return sets


def _nonzero_bytes(torch, f):
    torch.cuda.synchronize()
    ptr, nbytes = f.device_bits()

    class _B:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}

    t = torch.as_tensor(_B(), device="cuda")
    pos, val = [], []
    for a in range(0, nbytes, 1 << 28):   # torch.nonzero's scratch grows with its input: 256 MiB pieces
        nz = torch.nonzero(t[a: a + (1 << 28)]).view(-1) + a
        pos.append(nz.cpu().numpy())
        val.append(t[nz].cpu().numpy())
    return np.concatenate(pos), np.concatenate(val)


def _want_sparse(idx):
    u = np.unique(np.asarray(idx, np.uint64).reshape(-1))
    pos = (u >> np.uint64(3)).astype(np.int64)
    mask = (np.uint64(0x80) >> (u & np.uint64(7))).astype(np.uint8)
    if not len(u):
        return pos, mask
    st = np.flatnonzero(np.concatenate([[True], pos[1:] != pos[:-1]]))
    return pos[st], np.bitwise_or.reduceat(mask, st)


@pytest.mark.parametrize("rl", ["19", "18"])
@pytest.mark.parametrize("m,k,n", [
    (9585058, 6, 40_000),           # 1M@1 %: 19 regions, dense (bitmap and low-l sets)
    (1437758757, 10, 20_000),       # 100M@0.1 %: sparse, large l
    (9585058377, 6, 200_000),       # the north-star filter
    (191701167547, 13, 100_000),    # 10B@0.01 % (reach-capped 6.98 GB): 106k regions
])
def test_encoded_sets_equal_oracle_offsets(pkg, oracle, monkeypatch, rl, m, k, n):
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("BFHIP_BIN_REGION_LOG2", rl)
    rng = np.random.default_rng(SEED + k + int(rl))
    buf, offs = _keys(pkg, rng, n)
    idx = oracle.indexes_many(buf, offs, m, k)
    with pkg.Filter(m, k) as f:
        for digests in (False, True):
            sets = _encode(torch, f, buf, offs, digests=digests)
            words = sets.cpu().numpy().view(np.uint32)
            magic, got_rl, R, used = sets_codec.header(words)
            want_rl = int(rl) if (f.device_bytes * 8) >> int(rl) <= 131072 else 19   # 2^18 regions past 131072: 2^19
            assert (magic, got_rl) == (sets_codec.MAGIC, want_rl) and used <= len(words)
            assert abs(f.region_sets_capacity(n) - 4 * sets_codec.capacity_words(f.device_bytes, got_rl, n, k)) <= 256
            want = sets_codec.expected(idx, got_rl)
            got = sets_codec.decode(words)
            assert sorted(got) == sorted(want)
            for r in want:
                np.testing.assert_array_equal(got[r], want[r])


def test_bitmap_and_empty_sets(pkg, oracle):
    """A region hit by most of its offsets is written as its bitmap; an empty batch is a valid
    empty buffer (every region absent)."""
    torch = pytest.importorskip("torch")
    m, k = 1 << 20, 6   # two 2^19-bit regions
    rng = np.random.default_rng(SEED)
    buf, offs = _keys(pkg, rng, 300_000)
    with pkg.Filter(m, k) as f:
        words = _encode(torch, f, buf, offs).cpu().numpy().view(np.uint32)
        hdrs = [int(words[int(words[4 + r])]) >> 24 for r in range(2)]
        assert hdrs == [31, 31]
        want = sets_codec.expected(oracle.indexes_many(buf, offs, m, k), 19)
        got = sets_codec.decode(words)
        for r in want:
            np.testing.assert_array_equal(got[r], want[r])
        empty = _encode(torch, f, buf[:0], offs[:1]).cpu().numpy().view(np.uint32)
        assert sets_codec.decode(empty) == {}


@pytest.mark.parametrize("m,k,n", [
    (9585058, 6, 30_000),
    (1437758757, 10, 30_000),
    (9585058377, 6, 100_000),
    (191701167547, 13, 60_000),
])
def test_insert_sets_equals_inserting_the_keys(pkg, oracle, m, k, n):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(SEED + 7 * k)
    batches = [_keys(pkg, rng, n, "a"), _keys(pkg, rng, n // 3, "b"), _keys(pkg, rng, 0, "c"), _keys(pkg, rng, n, "d")]
    with pkg.Filter(m, k) as f:
        cap = max(f.region_sets_capacity(len(o) - 1) for _, o in batches)
        sets = torch.cat([_encode(torch, f, b, o, cap=cap) for b, o in batches])
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        probes = sum(len(o) - 1 for _, o in batches) * k
        f.insert_region_sets_dev(sets.data_ptr(), cap, len(batches), probes, d_any_new=flag.data_ptr(),
                                 d_status=status.data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert int(flag.item()) == 1 and int(status.item()) == 0
        idx = np.concatenate([oracle.indexes_many(b, o, m, k).reshape(-1) for b, o in batches])
        got_p, got_v = _nonzero_bytes(torch, f)
        want_p, want_v = _want_sparse(idx)
        np.testing.assert_array_equal(got_p, want_p)
        np.testing.assert_array_equal(got_v, want_v)
        # the same sets again change nothing: any_new stays 0 (every probe hits a set bit)
        flag.zero_()
        f.insert_region_sets_dev(sets.data_ptr(), cap, len(batches), probes, d_any_new=flag.data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert int(flag.item()) == 0


@pytest.mark.parametrize("m,k", [(9585058, 6), (9585058377, 6)])
def test_insert_sets_into_prefilled_filter_and_include(pkg, oracle, m, k):
    """OR into a filter already holding bits (a Redis string imported), then include? answers
    and the exported string equal the oracle's insert of the same keys into that string."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(SEED + 99)
    pre_b, pre_o = _keys(pkg, rng, 20_000, "p")
    batches = [_keys(pkg, rng, 25_000, "x%d" % s) for s in range(5)]
    with pkg.Filter(m, k) as f:
        f.insert_many(pre_b, pre_o)
        cap = f.region_sets_capacity(25_000)
        sets = torch.cat([_encode(torch, f, b, o, cap=cap) for b, o in batches])
        f.insert_region_sets_dev(sets.data_ptr(), cap, len(batches), 5 * 25_000 * k, stream=0)
        torch.cuda.synchronize()
        probe_b, probe_o = _keys(pkg, rng, 5_000, "x2")
        got_inc = f.include_many(probe_b, probe_o)
        got_s = f.export_redis() if m < 10**8 else None
    if m < 10**8:
        bits = oracle.new_bitset(m, k)
        oracle.insert_many(bits, m, k, pre_b, pre_o)
        for b, o in batches:
            oracle.insert_many(bits, m, k, b, o)
        assert got_s == oracle.redis_string(bits)
        np.testing.assert_array_equal(got_inc, oracle.include_many(bits, m, k, probe_b, probe_o))
    else:
        idx = np.concatenate([oracle.indexes_many(b, o, m, k).reshape(-1) for b, o in [(pre_b, pre_o)] + batches])
        pidx = oracle.indexes_many(probe_b, probe_o, m, k)
        want = np.isin(pidx, np.unique(idx)).all(axis=1)
        np.testing.assert_array_equal(got_inc.astype(bool), want)


@pytest.mark.parametrize("m,k,n", [(9585058377, 6, 100_000), (191701167547, 13, 60_000), (9585058, 6, 30_000)])
def test_insert_encode_equals_the_two_calls(pkg, oracle, m, k, n):
    """bf_insert_encode_region_sets_dev (the apply of one step's sets and the encode of the next
    batch in one kernel) against the two calls: the same bitset (checked against the oracle too),
    the same any_new and status, and a next-batch buffer whose sets decode to the oracle's
    offsets (tests/sets_codec.py) exactly as the separate encode's."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(SEED + 31 * k)
    batches = [_keys(pkg, rng, n, "p%d" % s) for s in range(3)]
    nb, no = _keys(pkg, rng, n, "next")
    with pkg.Filter(m, k) as fa, pkg.Filter(m, k) as fb:
        cap = fa.region_sets_capacity(n)
        sets = torch.cat([_encode(torch, fa, b, o, cap=cap) for b, o in batches])
        kb, ko = _dev(torch, nb, no)
        dig = torch.empty((n, 4), dtype=torch.int32, device="cuda")
        fa.hash_many_dev(kb.data_ptr(), ko.data_ptr(), n, dig.data_ptr(), stream=0)
        probes = 3 * n * k
        flags = torch.zeros(2, dtype=torch.int32, device="cuda")
        status = torch.zeros(2, dtype=torch.int32, device="cuda")
        nxt_a = torch.zeros(cap // 4, dtype=torch.int32, device="cuda")
        nxt_b = torch.zeros(cap // 4, dtype=torch.int32, device="cuda")
        fa.encode_region_sets_digests_dev(dig.data_ptr(), n, nxt_a.data_ptr(), cap, stream=0)
        fa.insert_region_sets_dev(sets.data_ptr(), cap, 3, probes, d_any_new=flags[0:].data_ptr(),
                                  d_status=status[0:].data_ptr(), stream=0)
        fb.insert_encode_region_sets_dev(sets.data_ptr(), cap, 3, probes, dig.data_ptr(), n, nxt_b.data_ptr(), cap,
                                         d_any_new=flags[1:].data_ptr(), d_status=status[1:].data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert flags.tolist() == [1, 1] and status.tolist() == [0, 0]
        pa, va = _nonzero_bytes(torch, fa)
        pb, vb = _nonzero_bytes(torch, fb)
        np.testing.assert_array_equal(pa, pb)
        np.testing.assert_array_equal(va, vb)
        idx = np.concatenate([oracle.indexes_many(b, o, m, k).reshape(-1) for b, o in batches])
        want_p, want_v = _want_sparse(idx)
        np.testing.assert_array_equal(pb, want_p)
        np.testing.assert_array_equal(vb, want_v)
        words = int(nxt_a[3].item())
        assert words == int(nxt_b[3].item())
        np.testing.assert_array_equal(nxt_a[:words].cpu().numpy(), nxt_b[:words].cpu().numpy())
        # and that buffer inserts the next batch: both filters take it and stay equal to the oracle
        fb.insert_region_sets_dev(nxt_b.data_ptr(), cap, 1, n * k, stream=0)
        pb2, vb2 = _nonzero_bytes(torch, fb)
        want_p2, want_v2 = _want_sparse(np.concatenate([idx, oracle.indexes_many(nb, no, m, k).reshape(-1)]))
        np.testing.assert_array_equal(pb2, want_p2)
        np.testing.assert_array_equal(vb2, want_v2)
        # the next buffer may not overlap the buffers it is applied with
        with pytest.raises(pkg.ArgumentError, match="overlaps"):
            fb.insert_encode_region_sets_dev(sets.data_ptr(), cap, 3, probes, dig.data_ptr(), n,
                                             sets[cap // 4:].data_ptr(), cap, stream=0)


@pytest.mark.parametrize("nsrc,n_next", [(17, 4000), (2, 0)])
def test_insert_encode_other_shapes(pkg, oracle, nsrc, n_next):
    """bf_insert_encode_region_sets_dev where the one-kernel form does not apply: 17 sources (more
    than one apply launch takes: the two calls run instead) and an empty next batch (its buffer is
    the header alone).  The bitset equals the oracle's, the next buffer inserts its batch."""
    torch = pytest.importorskip("torch")
    m, k = 9585058377, 6
    rng = np.random.default_rng(SEED + 61 + nsrc)
    batches = [_keys(pkg, rng, 3000, "q%d" % s) for s in range(nsrc)]
    nb, no = _keys(pkg, rng, n_next, "nx")
    with pkg.Filter(m, k) as f:
        cap = f.region_sets_capacity(max(3000, n_next))
        sets = torch.cat([_encode(torch, f, b, o, cap=cap) for b, o in batches])
        dig = torch.zeros((max(n_next, 1), 4), dtype=torch.int32, device="cuda")
        if n_next:
            kb, ko = _dev(torch, nb, no)
            f.hash_many_dev(kb.data_ptr(), ko.data_ptr(), n_next, dig.data_ptr(), stream=0)
        nxt = torch.zeros(cap // 4, dtype=torch.int32, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        f.insert_encode_region_sets_dev(sets.data_ptr(), cap, nsrc, nsrc * 3000 * k, dig.data_ptr(), n_next,
                                        nxt.data_ptr(), cap, d_status=status.data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert int(status.item()) == 0
        idx = np.concatenate([oracle.indexes_many(b, o, m, k).reshape(-1) for b, o in batches])
        got_p, got_v = _nonzero_bytes(torch, f)
        want_p, want_v = _want_sparse(idx)
        np.testing.assert_array_equal(got_p, want_p)
        np.testing.assert_array_equal(got_v, want_v)
        f.insert_region_sets_dev(nxt.data_ptr(), cap, 1, max(n_next, 1) * k, d_status=status.data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert int(status.item()) == 0
        if n_next:
            idx = np.concatenate([idx, oracle.indexes_many(nb, no, m, k).reshape(-1)])
        got_p, got_v = _nonzero_bytes(torch, f)
        want_p, want_v = _want_sparse(idx)
        np.testing.assert_array_equal(got_p, want_p)
        np.testing.assert_array_equal(got_v, want_v)


@pytest.mark.parametrize("m,k,n", [(9585058377, 6, 200_000), (191701167547, 13, 100_000)])
def test_encoder_handle_writes_the_same_sets(pkg, m, k, n):
    """An encoder handle (BF_FLAG_ENCODER) encodes with a persistent grid on part of the CUs
    (it runs beside another stream's apply); its buffer is word for word the filter handle's."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(SEED + 71 + k)
    b, o = _keys(pkg, rng, n, "enc")
    with pkg.Filter(m, k) as f, pkg.Filter(m, k, flags=pkg._lib.BF_FLAG_ENCODER) as enc:
        cap = f.region_sets_capacity(n)
        assert enc.region_sets_capacity(n) == cap
        kb, ko = _dev(torch, b, o)
        dig = torch.empty((n, 4), dtype=torch.int32, device="cuda")
        f.hash_many_dev(kb.data_ptr(), ko.data_ptr(), n, dig.data_ptr(), stream=0)
        sa = torch.zeros(cap // 4, dtype=torch.int32, device="cuda")
        sb = torch.zeros(cap // 4, dtype=torch.int32, device="cuda")
        f.encode_region_sets_digests_dev(dig.data_ptr(), n, sa.data_ptr(), cap, stream=0)
        enc.encode_region_sets_digests_dev(dig.data_ptr(), n, sb.data_ptr(), cap, stream=0)
        torch.cuda.synchronize()
        words = int(sa[3].item())
        assert words == int(sb[3].item()) and words > 4
        np.testing.assert_array_equal(sa[:words].cpu().numpy(), sb[:words].cpu().numpy())


def test_foreign_set_buffer_is_skipped(pkg):
    """A buffer encoded for another filter size does not match this filter's regions: it is
    skipped (no bit set) and d_status flags it; the ABI refuses a short capacity."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(SEED + 5)
    buf, offs = _keys(pkg, rng, 10_000)
    with pkg.Filter(1437758757, 10) as other, pkg.Filter(9585058, 6) as f:
        sets = _encode(torch, other, buf, offs)
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        cap = sets.numel() * 4
        f.insert_region_sets_dev(sets.data_ptr(), cap, 1, 60_000, d_status=status.data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert int(status.item()) == 1 and f.export_redis() == b""
        kb, ko = _dev(torch, buf, offs)
        small = torch.zeros(64, dtype=torch.int32, device="cuda")
        with pytest.raises(pkg.ArgumentError):
            f.encode_region_sets_dev(kb.data_ptr(), ko.data_ptr(), 10_000, small.data_ptr(), 256, stream=0)


def test_damaged_region_entry_is_skipped(pkg, oracle):
    """A region whose table entry points past its buffer, or whose header is not a set shape
    (l past the region size; an Elias-Fano set with l = 0, which the encoder never writes),
    is skipped and flagged; every other region of the buffer is applied as encoded."""
    torch = pytest.importorskip("torch")
    m, k = 9585058377, 6
    rng = np.random.default_rng(SEED + 11)
    buf, offs = _keys(pkg, rng, 50_000)
    idx = oracle.indexes_many(buf, offs, m, k)
    with pkg.Filter(m, k) as f:
        sets = _encode(torch, f, buf, offs)
        words = sets.cpu().numpy().view(np.uint32).copy()
        _, rl, R, _ = sets_codec.header(words)
        want = sets_codec.expected(idx, rl)
        bad = sorted(want)[:3]
        words[4 + bad[0]] = len(words) - 2            # a place whose set runs past the buffer
        words[4 + R + bad[1]] = (1 << 24) | (25 << 24)   # l = 26 > region_log2: not a set shape
        words[4 + R + bad[2]] &= 0xFFFFFF                # l = 0: not an Elias-Fano set shape
        damaged = torch.from_numpy(words.view(np.int32)).cuda()
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        f.insert_region_sets_dev(damaged.data_ptr(), damaged.numel() * 4, 1, 50_000 * k,
                                 d_status=status.data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert int(status.item()) == 1
        got = np.frombuffer(f.export_redis(), np.uint8)
        exp_bits = np.concatenate([(np.uint64(r) << np.uint64(rl)) + want[r] for r in want if r not in bad])
        expect = np.zeros(len(got), np.uint8)
        np.bitwise_or.at(expect, (exp_bits >> np.uint64(3)).astype(np.int64),
                         (np.uint8(0x80) >> (exp_bits & np.uint64(7)).astype(np.uint8)))
        np.testing.assert_array_equal(got, expect[: len(got)])


@pytest.mark.parametrize("nsrc", [17, 33])
def test_many_sources_take_several_launches(pkg, oracle, nsrc):
    """More sources than one sets_apply launch takes (kMaxSetSrc = 16): the sources go in 16
    at a time, and the bitset equals the oracle's insert of every batch."""
    torch = pytest.importorskip("torch")
    m, k = 9585058, 6
    rng = np.random.default_rng(SEED + nsrc)
    batches = [_keys(pkg, rng, 3_000 + 97 * s, "m%d" % s) for s in range(nsrc)]
    with pkg.Filter(m, k) as f:
        cap = max(f.region_sets_capacity(len(o) - 1) for _, o in batches)
        sets = torch.cat([_encode(torch, f, b, o, cap=cap) for b, o in batches])
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        probes = sum(len(o) - 1 for _, o in batches) * k
        f.insert_region_sets_dev(sets.data_ptr(), cap, nsrc, probes, d_any_new=flag.data_ptr(),
                                 d_status=status.data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert int(status.item()) == 0 and int(flag.item()) == 1
        got = f.export_redis()
    bits = oracle.new_bitset(m, k)
    for b, o in batches:
        oracle.insert_many(bits, m, k, b, o)
    assert got == oracle.redis_string(bits)


def test_sets_api_refusals(pkg):
    """a stride shorter than a buffer's header and tables, an engine filter (the
    sets carry the ruby driver's offsets), and a batch one encode cannot take (no capacity is
    given for it, so every rank that sizes its buffers from the largest batch learns it) are
    refused; a buffer whose reserved-words field does not cover its own tables is skipped."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(SEED + 21)
    buf, offs = _keys(pkg, rng, 5_000)
    m, k = 9585058377, 6
    with pkg.Filter(m, k) as f:
        sets = _encode(torch, f, buf, offs)
        words = sets.cpu().numpy().view(np.uint32)
        R = int(words[2])
        first = (4 + 2 * R + 63) // 64 * 64
        with pytest.raises(pkg.ArgumentError):
            f.insert_region_sets_dev(sets.data_ptr(), 4 * (R + 4), 1, 30_000, stream=0)
        with pytest.raises(pkg.ArgumentError):
            f.region_sets_capacity(1 << 34)
        bad = words.copy()
        bad[3] = first - 1
        damaged = torch.from_numpy(bad.view(np.int32)).cuda()
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        f.insert_region_sets_dev(damaged.data_ptr(), damaged.numel() * 4, 1, 30_000, d_status=status.data_ptr(),
                                 stream=0)
        torch.cuda.synchronize()
        assert int(status.item()) == 1 and f.export_redis() == b""
    with pkg.Filter(m, k, flags=pkg.BF_FLAG_ENGINE_MD5) as e:
        with pytest.raises(pkg.ArgumentError):
            e.insert_region_sets_dev(sets.data_ptr(), sets.numel() * 4, 1, 30_000, stream=0)
        with pytest.raises(pkg.ArgumentError):
            e.region_sets_capacity(1000)

