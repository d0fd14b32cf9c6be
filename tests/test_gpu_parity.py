"""HIP path vs the CPU oracle, through the C ABI (libbfhip.so).

Bit-exact: the k offsets of every key, the Redis string after a fixed insert
sequence, and every include? answer, against oracle/ (the restatement of
lib/bloomfilter_driver/ruby.rb:41-63 and lib/redis/bloomfilter.rb:50-58).
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RNG_SEED = 0x5EED


def rand_keys(rng, n, lo=0, hi=200):
    lens = rng.integers(lo, hi + 1, size=n)
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    buf = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    return buf, offs


def w8_keys(rng, n):
    """bf_10_000.rb:8-11 family: 8 distinct lowercase letters."""
    letters = np.argsort(rng.random((n, 26)), axis=1)[:, :8].astype(np.uint8) + ord("a")
    buf = letters.reshape(-1).copy()
    offs = np.arange(0, 8 * n + 1, 8, dtype=np.uint64)
    return buf, offs


def edge_keys():
    """Every length across the SHA-1 block boundaries (55/56, 63/64, 119/120 ...)."""
    keys = [bytes((i * 7 + j) & 0xFF for j in range(L)) for i, L in enumerate(range(0, 260))]
    keys += ["asdlol", "foo", "", "héllo wörld ✓", "a" * 55, "b" * 56, "c" * 64, "d" * 119, "e" * 120]
    keys += [str(i) for i in (0, 42, 999, 10**9, 2**63)]
    return keys


REGIMES = [
    (9585, 6),                     # spec 1000@1% (spec:56-57)
    (95851, 6),                    # 10k@1%
    (95851, 7),
    (1, 1),
    (2, 3),
    (9585058, 6),                  # 1M@1%
    (1437758757, 10),              # 100M@0.1%
    (2**32 + 17, 10),              # 2^32 <= m < k*2^32
    (9585058377, 6),               # 1B@1% (north star)
    (13 * 0xFFFFFFFF + 1, 13),     # m == reach (largest m still reduced)
    (191701167547, 13),            # 10B@0.01%: m > k*(2^32-1), modulo skipped
    (3834023350947, 13),           # 200B@0.01% (BASELINE configs[4]): modulo skipped, same reach
    (2**40 + 3, 64),               # k = BF_MAX_K
    # float32-quotient modulo boundaries (m >= 2^17) and the float64 path below it
    (2**17 - 1, 13), (2**17, 13), (2**17 + 1, 64), (2**32 - 1, 13), (2**32, 6), (2**32 + 1, 64),
    (999999999989, 64), (3, 64), (131071 * 7, 9),
]


@pytest.mark.parametrize("m,k", REGIMES)
def test_indexes_match_oracle(pkg, oracle, m, k):
    rng = np.random.default_rng(RNG_SEED + k)
    buf, offs = rand_keys(rng, 3000)
    e_buf, e_offs = pkg.keys.pack(edge_keys())
    with pkg.Filter(m, k) as f:
        for b, o in ((buf, offs), (e_buf, e_offs)):
            got = f.indexes_many(b, o)
            want = oracle.indexes_many(b, o, m, k)
            assert got.shape == want.shape
            np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("m,k", [(9585, 6), (2**32 + 17, 10), (191701167547, 13), (2**40 + 3, 64)])
def test_single_key_indexes_no_filter(pkg, oracle, m, k):
    """bf_indexes (handle-free, one key): the same device kernel, no bitset allocated —
    so the 10B / 2^40-bit regimes cost nothing here."""
    for key in ["asdlol", "", "a" * 55, "b" * 56, "d" * 119, "héllo wörld ✓", "42"]:
        b, o = pkg.keys.pack([key])
        want = oracle.indexes_many(b, o, m, k).reshape(-1).tolist()
        assert pkg._lib.indexes(bytes(b), m, k) == want


def test_known_answers(pkg):
    """SURVEY §7 known answers (Python hashlib + Node crypto restatements)."""
    cases = {("asdlol", 9585, 6): [5260, 6438, 144, 8807, 5008, 5791],
             ("foo", 95851, 7): [61181, 74832, 85954, 69596, 70715, 28527, 39649],
             (42, 9585, 6): [6198, 1190, 536, 3493, 2299, 9036],
             ("", 9585, 6): [8986, 4917, 7472, 7054, 4436, 1889]}
    for (key, m, k), want in cases.items():
        with pkg.Filter(m, k) as f:
            b, o = pkg.keys.pack([key])
            assert f.indexes_many(b, o)[0].tolist() == want


def _insert_include_roundtrip(pkg, oracle, m, k, ins, probe, **fkw):
    (ib, io), (pb, po) = ins, probe
    with pkg.Filter(m, k, **fkw) as f:
        f.insert_many(ib, io)
        got_str = f.export_redis()
        got_inc = f.include_many(pb, po)
    bits = oracle.new_bitset(m, k)
    oracle.insert_many(bits, m, k, ib, io)
    want_str = oracle.redis_string(bits)
    want_inc = oracle.include_many(bits, m, k, pb, po)
    assert len(got_str) == len(want_str)
    assert hashlib.sha1(got_str).hexdigest() == hashlib.sha1(want_str).hexdigest()
    np.testing.assert_array_equal(got_inc, want_inc)
    return got_str, got_inc


def test_spec_strings(pkg, oracle):
    """SURVEY §7 pinned strings: 'asdlol' alone; "0".."999" into 1000@1%."""
    s, _ = _insert_include_roundtrip(pkg, oracle, 9585, 6, pkg.keys.pack(["asdlol"]),
                                     pkg.keys.pack(["asdlol", "nope"]))
    assert len(s) == 1101
    assert hashlib.sha1(s).hexdigest() == "fdb117fe21dea15cb79ef9decc983623b10f8af9"
    s, _ = _insert_include_roundtrip(pkg, oracle, 9585, 6, pkg.keys.pack([str(i) for i in range(1000)]),
                                     pkg.keys.pack([str(i) for i in range(2000)]))
    assert len(s) == 1198
    assert hashlib.sha1(s).hexdigest() == "5e73e7002948f579501e9a6577af1f9c2c5364f3"
    assert sum(bin(x).count("1") for x in s) == 4438


def test_config_10k_w8(pkg, oracle):
    rng = np.random.default_rng(RNG_SEED)
    ins = w8_keys(rng, 10_000)
    probe = w8_keys(rng, 20_000)
    _, inc = _insert_include_roundtrip(pkg, oracle, 95851, 6, ins, probe)
    assert 0 < inc.sum() < len(inc)


def test_config_1m_decimal(pkg, oracle):
    rng = np.random.default_rng(RNG_SEED + 1)
    vals = rng.integers(0, 10**6, size=10**6)
    ins = pkg.keys.pack_decimal(vals)
    probe = pkg.keys.pack_decimal(np.concatenate([vals[:500_000], rng.integers(10**6, 2 * 10**6, 500_000)]))
    _, inc = _insert_include_roundtrip(pkg, oracle, 9585058, 6, ins, probe)
    assert inc[:500_000].all()   # no false negatives


def test_long_keys_fallback_and_chunking(pkg, oracle):
    """Workgroup spans > 16 KiB take the global-read path; tiny host chunks force many chunks."""
    rng = np.random.default_rng(RNG_SEED + 2)
    ins = rand_keys(rng, 3000, 50, 400)
    probe = rand_keys(rng, 3000, 0, 400)
    ib, io = ins
    probe = (np.concatenate([ib, probe[0]]), np.concatenate([io, probe[1][1:] + io[-1]]))
    _insert_include_roundtrip(pkg, oracle, 95851, 7, ins, probe)
    _insert_include_roundtrip(pkg, oracle, 95851, 7, ins, probe, batch_keys=257, batch_bytes=5000)


def test_offsets_not_starting_at_zero(pkg, oracle):
    rng = np.random.default_rng(RNG_SEED + 3)
    buf, offs = rand_keys(rng, 1000, 0, 40)
    sub_offs = offs[100:]   # keys 100.. of the same buffer
    with pkg.Filter(95851, 6) as f:
        np.testing.assert_array_equal(f.indexes_many(buf, sub_offs),
                                      oracle.indexes_many(buf, sub_offs, 95851, 6))


def test_empty_and_single(pkg):
    with pkg.Filter(9585, 6) as f:
        b, o = pkg.keys.pack([])
        assert f.include_many(b, o).shape == (0,)
        any_new, _ = f.insert_many(b, o, any_new=True)
        assert any_new is False
        assert f.export_redis() == b""
        b, o = pkg.keys.pack([""])
        any_new, pk = f.insert_many(b, o, any_new=True, per_key_new=True)
        assert any_new is True and pk.tolist() == [1]
        assert f.include_many(b, o).tolist() == [1]


def test_any_new_and_per_key(pkg, oracle):
    rng = np.random.default_rng(RNG_SEED + 4)
    b, o = pkg.keys.pack_decimal(rng.permutation(10**6)[:5000])
    with pkg.Filter(9585058377, 6) as f:   # sparse: no intra-batch collisions expected
        any_new, pk = f.insert_many(b, o, any_new=True, per_key_new=True)
        assert any_new is True and pk.all()
        any_new, pk = f.insert_many(b, o, any_new=True, per_key_new=True)
        assert any_new is False and not pk.any()
    with pkg.Filter(9585, 6) as f:           # dense: per-key flags follow the keys' order exactly
        b, o = pkg.keys.pack([str(i) for i in range(3000)])
        any_new, pk = f.insert_many(b, o, any_new=True, per_key_new=True)
        bits = oracle.new_bitset(9585, 6)
        seq_any, seq_pk = oracle.insert_many(bits, 9585, 6, b, o, per_key=True)
        assert any_new == seq_any
        np.testing.assert_array_equal(pk, seq_pk)
        assert f.export_redis() == oracle.redis_string(bits)


@pytest.mark.parametrize("m,k,n,chunk", [(9585, 6, 5000, 0), (95851, 7, 40_000, 0), (95851, 7, 40_000, 997),
                                         (2**32 + 17, 13, 20_000, 0), (9585058377, 6, 100_000, 0),
                                         (1000, 64, 300, 0), (70001, 64, 6000, 0), (2**27, 7, 50_000, 0)])
def test_per_key_new_is_sequential(pkg, oracle, m, k, n, chunk):
    """per_key_new[j] == 1 iff inserting the batch key by key (ruby.rb:57-61), key j flipped a
    bit: exact against the oracle's sequential loop, with repeated keys, dense filters
    (many keys sharing bits within the batch), host chunks (batch_keys) and a prefilled filter.
    Batches of 4096+ keys on filters of up to 2^27 bits take the binned form (bf_seq.hip: the
    first-index table per 2^14-bit region in LDS): 9585 / 95851 (a partial last region) / 70001
    at k = 64 / 2^27 (8192 regions, the form's limit); the others the direct or hash forms."""
    rng = np.random.default_rng(RNG_SEED + 9)
    vals = rng.integers(0, n // 2, size=n)                 # ~half the batch repeats earlier keys
    b, o = pkg.keys.pack_decimal(vals)
    pre_b, pre_o = pkg.keys.pack_decimal(rng.integers(10**6, 2 * 10**6, size=n // 4))
    bits = oracle.new_bitset(m, k)
    oracle.insert_many(bits, m, k, pre_b, pre_o)
    want_any, want_pk = oracle.insert_many(bits, m, k, b, o, per_key=True)
    with pkg.Filter(m, k, batch_keys=chunk) as f:
        f.insert_many(pre_b, pre_o)
        any_new, pk = f.insert_many(b, o, any_new=True, per_key_new=True)
        np.testing.assert_array_equal(pk, want_pk)
        assert any_new == bool(want_any)
        assert f.export_redis() == oracle.redis_string(bits)


def test_spec_error_rate_as_one_batch(pkg, oracle):
    """spec/redis_bloomfilter_spec.rb:7-17 (test_error_rate) and bf_10_000.rb:34-43 ask include?
    before each insert; found-before-insert is !per_key_new, so one batched call reproduces the
    per-key loop's error count exactly."""
    rng = np.random.default_rng(RNG_SEED + 10)
    elems = 180
    vals = rng.integers(0, elems, size=elems)
    b, o = pkg.keys.pack_decimal(vals)
    m = pkg.Bloomfilter.optimal_m(100, 0.02)
    k = pkg.Bloomfilter.optimal_k(100, m)
    with pkg.Filter(m, k) as f:
        _, pk = f.insert_many(b, o, per_key_new=True)
    found = pk == 0
    bits = oracle.new_bitset(m, k)
    visited, errors, want_errors = set(), 0, 0
    for j, v in enumerate(vals.tolist()):
        kb, ko = pkg.keys.pack([v])
        seq_found = bool(oracle.include_many(bits, m, k, kb, ko)[0])
        oracle.insert_many(bits, m, k, kb, ko)
        assert found[j] == seq_found
        errors += found[j] != (v in visited)
        want_errors += seq_found != (v in visited)
        visited.add(v)
    assert errors == want_errors
    assert round(errors / elems, 2) <= 0.02                # spec:104


def test_import_export(pkg, oracle):
    rng = np.random.default_rng(RNG_SEED + 5)
    ib, io = rand_keys(rng, 2000, 0, 30)
    bits = oracle.new_bitset(95851, 6)
    oracle.insert_many(bits, 95851, 6, ib, io)
    s = oracle.redis_string(bits)
    with pkg.Filter(95851, 6) as f:
        f.import_redis(s)
        assert f.export_redis() == s
        np.testing.assert_array_equal(f.include_many(ib, io), np.ones(2000, np.uint8))
        # OR mode: union with a second string
        jb, jo = rand_keys(rng, 500, 0, 30)
        bits2 = oracle.new_bitset(95851, 6)
        oracle.insert_many(bits2, 95851, 6, jb, jo)
        f.import_redis(oracle.redis_string(bits2), mode=1)
        union = np.bitwise_or(bits, bits2)
        assert f.export_redis() == oracle.redis_string(union)
        # strings reaching past m are rejected (the ruby driver never writes them)
        with pytest.raises(pkg.ArgumentError):
            f.import_redis(b"\x00" * ((95851 + 7) // 8) + b"\x01")
        with pytest.raises(pkg.ArgumentError):
            f.import_redis(b"\x00" * ((95851 + 7) // 8 - 1) + b"\xff")   # bits >= m in the last byte
        f.clear()
        assert f.export_redis() == b""


def test_device_api_torch(pkg, oracle):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(RNG_SEED + 6)
    buf, offs = rand_keys(rng, 4097, 0, 70)
    dk = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    m, k = 1437758757, 10
    st = torch.cuda.current_stream().cuda_stream
    with pkg.Filter(m, k) as f:
        idx = torch.empty((4097, k), dtype=torch.int64, device="cuda")
        f.indexes_many_dev(dk.data_ptr(), do.data_ptr(), 4097, idx.data_ptr(), stream=st)
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        f.insert_many_dev(dk.data_ptr(), do.data_ptr(), 4097, flag.data_ptr(), stream=st)
        out = torch.empty(4097, dtype=torch.uint8, device="cuda")
        f.include_many_dev(dk.data_ptr(), do.data_ptr(), 4097, out.data_ptr(), stream=st)
        f.sync()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint64), oracle.indexes_many(buf, offs, m, k))
        assert int(flag.item()) == 1
        assert out.cpu().numpy().all()
        # unaligned device key pointer (offset 3 bytes into the buffer)
        dk2 = torch.zeros(len(buf) + 3, dtype=torch.uint8, device="cuda")
        dk2[3:] = dk
        f.indexes_many_dev(dk2.data_ptr() + 3, do.data_ptr(), 4097, idx.data_ptr(), stream=st)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint64), oracle.indexes_many(buf, offs, m, k))


@pytest.mark.parametrize("mode", ["0", "1"])
@pytest.mark.parametrize("m,k,n", [(95851, 6, 20_000), (9585058, 6, 300_000), (1437758757, 10, 200_000),
                                   (2**32 + 17, 7, 100_000), (95851, 6, 1_500_000)])
def test_binned_insert_matches_oracle(pkg, oracle, monkeypatch, mode, m, k, n):
    """BFHIP_INSERT_BINNED / BFHIP_INCLUDE_BINNED = 1 force the binned (front/mid/apply|test)
    insert and include?; 0 the direct kernels.  1.5M keys into one region: a superbin of more
    than one run-table pass (> 1024 chunk blocks) and a region of many probe steps."""
    monkeypatch.setenv("BFHIP_INSERT_BINNED", mode)
    monkeypatch.setenv("BFHIP_INCLUDE_BINNED", mode)
    rng = np.random.default_rng(RNG_SEED + 7)
    ins = rand_keys(rng, n, 0, 24)
    probe = rand_keys(rng, 20_000, 0, 24)
    ib, io = ins
    probe = (np.concatenate([ib, probe[0]]), np.concatenate([io[:5001], probe[1][1:] + io[-1]]))
    s, _ = _insert_include_roundtrip(pkg, oracle, m, k, ins, probe)
    with pkg.Filter(m, k) as f:                       # any_new through the binned path
        any1, _ = f.insert_many(ib, io, any_new=True)
        any2, _ = f.insert_many(ib, io, any_new=True)
        assert (any1, any2) == (True, False)
        assert f.export_redis() == s


# Every case at every region size: 2^19 bits (the default), and the 2^18 / 2^20 templates
# (512-lane apply / test, 128 KiB LDS images) — ADVICE r04: the DPP block scan, the apply's
# XCD remap and LOADS template and the route fronts' compile-time slots reach all of them
# (the 10B filter at 2^18 takes 2^19, so k13 runs at 19 and 20 only)
EDGE_CASES = ([("19", c) for c in ("dup", "tiny", "long", "k12", "k13", "k16", "nstar")] +
              [("18", c) for c in ("dup", "tiny", "long", "k12", "k16", "nstar")] +
              [("20", c) for c in ("dup", "tiny", "long", "k12", "k13", "k16", "nstar")])


@pytest.mark.parametrize("rl,case", EDGE_CASES)
def test_binned_edge_cases(pkg, oracle, monkeypatch, rl, case):
    """Forced binned insert and include? on shapes that stress their partition passes: one key repeated
    (every probe in <= k regions, one superbin run per tile holding thousands of probes),
    a few keys over the 1.2 GB north-star filter (a level-2 chunk spanning every superbin:
    the per-probe cursor path), keys past the single-block SHA-1 (multi-block hash in the
    count pass), k = 12 (every probe slot of the 12-slot front used), k = 13 and 16 (the 16-slot
    front), and a 200k-key batch on the
    north-star filter; every region size (32 / 64 / 128 KiB LDS images)."""
    monkeypatch.setenv("BFHIP_INSERT_BINNED", "1")
    monkeypatch.setenv("BFHIP_INCLUDE_BINNED", "1")
    monkeypatch.setenv("BFHIP_BIN_REGION_LOG2", rl)
    rng = np.random.default_rng(RNG_SEED + 8)
    if case == "dup":
        m, k = 1437758757, 10
        ins = pkg.keys.pack(["same-key"] * 60_000 + [str(i) for i in range(100)])
    elif case == "tiny":
        m, k = 9585058377, 6
        ins = rand_keys(rng, 37, 0, 20)
    elif case == "long":
        m, k = 1437758757, 6
        ins = rand_keys(rng, 20_000, 56, 300)
    elif case == "k12":
        m, k = 2**32 + 17, 12
        ins = rand_keys(rng, 30_000, 0, 24)
    elif case == "k13":   # 16 probe slots per lane from here (bin_front_wide_kernel)
        m, k = 191701167547, 13
        ins = rand_keys(rng, 30_000, 0, 24)
    elif case == "k16":
        m, k = 9585058377, 16
        ins = rand_keys(rng, 30_000, 0, 70)
    else:
        m, k = 9585058377, 6
        ins = pkg.keys.pack_decimal(rng.integers(0, 10**9, size=200_000))
    ib, io = ins
    extra = rand_keys(rng, 5_000, 0, 24)
    probe = (np.concatenate([ib, extra[0]]), np.concatenate([io, extra[1][1:] + io[-1]]))
    _insert_include_roundtrip(pkg, oracle, m, k, ins, probe)


@pytest.mark.parametrize("binned", ["0", "1"])
def test_config_200b(pkg, oracle, monkeypatch, binned):
    """BASELINE configs[4]'s filter, 200B keys @ 0.01 %: m = 3,834,023,350,947, k = 13.  m is far
    beyond k*(2^32-1), so ruby.rb:51's modulo never reduces and the offsets stay below
    k*(2^32-1)+1: the device holds that 6.98 GB reachable prefix (1.46 % of m).  Offsets,
    the Redis string (length + sha1) and include? answers against the oracle, through the
    direct and the binned insert."""
    monkeypatch.setenv("BFHIP_INSERT_BINNED", binned)
    m = pkg.Bloomfilter.optimal_m(2 * 10**11, 0.0001)
    k = pkg.Bloomfilter.optimal_k(2 * 10**11, m)
    assert (m, k) == (3834023350947, 13)
    rng = np.random.default_rng(RNG_SEED + 11)
    ins = pkg.keys.pack_decimal(rng.integers(0, 2 * 10**11, size=4000))
    probe = pkg.keys.pack_decimal(rng.integers(0, 2 * 10**11, size=4000))
    ib, io = ins
    pb, po = probe
    probe = (np.concatenate([ib, pb]), np.concatenate([io, po[1:] + io[-1]]))
    with pkg.Filter(m, k) as f:
        assert f.reach_bits == k * 0xFFFFFFFF + 1
        np.testing.assert_array_equal(f.indexes_many(ib, io), oracle.indexes_many(ib, io, m, k))
    s, inc = _insert_include_roundtrip(pkg, oracle, m, k, ins, probe)
    assert inc[:4000].all()
    assert len(s) * 8 <= k * 0xFFFFFFFF + 1
