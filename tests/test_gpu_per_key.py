"""The per-key (small-batch) host path: the latency path of bf_insert_many / bf_include_many
and bf_insert_many_changes, whose flipped-bit list is what the hip driver's write-through
replays as SETBITs (ruby.rb:57-63), checked against the oracle and against the Redis string
the ruby driver's restatement builds."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits_of(s: bytes):
    a = np.frombuffer(s, dtype=np.uint8)
    return set(np.flatnonzero(np.unpackbits(a)).tolist())   # MSB-first: bit o of byte o >> 3


@pytest.mark.parametrize("m,k", [(9585, 6), (95851, 6), (9585058, 6)])
def test_changes_are_the_flipped_bits(pkg, oracle, m, k):
    keys = ["k%d" % i for i in range(300)] + ["k7", "k7", ""]   # repeats: a bit flips once
    with pkg.Filter(m, k, device=0) as f:
        f.track_dirty(True)
        before = set()
        for lo in range(0, len(keys), 37):
            b, o = pkg.keys.pack(keys[lo: lo + 37])
            flips = f.insert_many_changes(b, o)
            after = _bits_of(f.export_redis())
            assert len(flips) == len(set(flips.tolist())), "a flipped bit was reported twice"
            assert set(flips.tolist()) == after - before
            before = after
        ib, io = pkg.keys.pack(keys)
        bits = oracle.new_bitset(m, k)
        oracle.insert_many(bits, m, k, ib, io)
        assert f.export_redis() == oracle.redis_string(bits)
        b, o = pkg.keys.pack(keys[:5])
        assert len(f.insert_many_changes(b, o)) == 0   # nothing new
        assert f.dirty_ranges(clear=False)[0] == []     # and the dirty map never marked


@pytest.mark.parametrize("m,k", [(1437758757, 10), (191701167547, 13), (3834023350947, 13)])
def test_changes_on_large_filters(pkg, oracle, m, k):
    """Offsets past 2^32 (the 10B / 200B filters' reach-capped 6.98e9 bits): on an empty
    filter the flipped bits are exactly the keys' distinct offsets (ruby.rb:41-55)."""
    keys = ["big-%d" % i for i in range(200)] + ["big-3"]
    b, o = pkg.keys.pack(keys)
    want = set()
    for key in keys:
        want.update(oracle.indexes(key, m, k))
    with pkg.Filter(m, k, device=0) as f:
        f.track_dirty(True)
        flips = f.insert_many_changes(b, o)
        assert sorted(flips.tolist()) == sorted(want)
        assert m < 1 << 32 or max(want) > 1 << 32
        assert f.dirty_ranges(clear=False)[0] == []


def test_changes_argument_limits(pkg):
    with pkg.Filter(95851, 6, device=0) as f:
        b, o = pkg.keys.pack(["x%d" % i for i in range(683)])   # 683 * 6 = 4098 > 4096 probes
        with pytest.raises(pkg.ArgumentError):
            f.insert_many_changes(b, o)
        b, o = pkg.keys.pack(["y" * 70000])                      # > 64 KiB of key bytes
        with pytest.raises(pkg.ArgumentError):
            f.insert_many_changes(b, o)
        b, o = pkg.keys.pack([])
        assert len(f.insert_many_changes(b, o)) == 0


@pytest.mark.parametrize("n", [1, 2, 17, 2048, 2049, 5000])
def test_small_and_pipelined_paths_agree(pkg, oracle, n):
    """Calls at, just past and well past the latency path's 2048-key limit give the oracle's
    answers, flags and string."""
    m, k = 9585058, 6
    rng = np.random.default_rng(n)
    ins = rng.integers(0, 10 ** 9, size=n)
    q = np.concatenate([ins[: n // 2], rng.integers(10 ** 9, 2 * 10 ** 9, size=n - n // 2)])
    ib, io = pkg.keys.pack(ins)
    qb, qo = pkg.keys.pack(q)
    with pkg.Filter(m, k, device=0) as f:
        any_new, per_key = f.insert_many(ib, io, any_new=True, per_key_new=True)
        bits = oracle.new_bitset(m, k)
        _, want_pk = oracle.insert_many(bits, m, k, ib, io, per_key=True)
        assert any_new is True
        assert np.array_equal(per_key, want_pk)
        assert f.export_redis() == oracle.redis_string(bits)
        assert np.array_equal(f.include_many(qb, qo), oracle.include_many(bits, m, k, qb, qo))
        any_new, _ = f.insert_many(ib, io, any_new=True)
        assert any_new is False


def test_write_through_setbits_match_ruby_driver(pkg, O):
    """Per-key inserts through the facade with write-through: the Redis string after every
    insert equals the ruby driver's (ruby.rb:57-63 over FakeRedis), and the device copy."""
    m = O.py_optimal_m(2000, 0.01)
    k = O.py_optimal_k(2000, m)
    r_hip, r_ref = pkg.FakeRedis(), pkg.FakeRedis()
    bf = pkg.Bloomfilter(size=2000, error_rate=0.01, key_name="wt", driver="hip", redis=r_hip)
    ref = O.RubyDriverRestatement({"bits": m, "hashes": k, "key_name": "wt", "redis": r_ref})
    for i in range(400):
        key = "word-%d" % (i % 350)
        got = bf.insert(key)
        ref.insert(key)
        assert r_hip.get("wt") == r_ref.get("wt"), i
        assert got == (i < 350)   # !found: fresh keys flip bits (no collisions at this size)
    assert bf.driver.to_redis_string() == r_ref.get("wt")
    assert bf.driver.filter.dirty_ranges(clear=False)[0] == []   # the SETBIT path leaves no dirty blocks
    bf.insert_many(["w%d" % i for i in range(2000)])              # a large batch: dirty-block flush
    assert r_hip.get("wt") == bf.driver.to_redis_string()
    bf.driver.close()


@pytest.mark.parametrize("engine", ["md5", "sha1"])
def test_write_through_setbits_ruby_test_engines(pkg, O, engine):
    """hip-test per-key write-through replays the engine kernel's flipped bits: the Redis
    string equals the RubyTest driver's SETBITs (ruby_test.rb:43-68) over the same keys."""
    m = O.py_optimal_m(500, 0.01)
    k = O.py_optimal_k(500, m)
    r = pkg.FakeRedis()
    bf = pkg.Bloomfilter(size=500, error_rate=0.01, key_name="rt", driver="hip-test", hash_engine=engine, redis=r)
    ref = O.PyBitstring()
    for i in range(150):
        key = "rt-%d" % (i % 120)
        changed = [ref.setbit(o, 1) for o in O.py_engine_indexes(key, m, k, engine)]
        got = bf.insert(key)
        assert got == (0 in changed), i
        assert r.get("rt") == ref.value(), i
    assert bf.driver.filter.dirty_ranges(clear=False)[0] == []
    bf.driver.close()


def test_write_through_batches_pick_the_cheaper_sync(pkg):
    """A 10k-key batch into the 180 MB (100M@0.1 %) string replays its flipped bits as SETBITs
    in bf_insert_many_changes-sized pieces (100k probes x 1 KB < the 180 MB block flush); a
    5k-key batch into a 12 KB string flushes dirty blocks.  Either way Redis ends equal to the
    device, and the replayed bits are each set once."""
    big = pkg.Bloomfilter(size=10 ** 8, error_rate=0.001, key_name="big", driver="hip", redis=pkg.FakeRedis())
    keys = np.random.default_rng(5).integers(0, 1 << 60, size=10000)
    assert big.driver._setbit_sync(pkg.keys.pack(keys)[1])
    assert big.insert_many(keys) is True
    r = big.redis
    calls = [c for c, _ in r.calls]
    assert "SETRANGE" not in calls and calls.count("SETBIT") > 50000
    assert r.get("big") == big.driver.to_redis_string()
    assert big.driver.filter.dirty_ranges(clear=False)[0] == []
    assert big.insert_many(keys) is False                        # nothing flips: no SETBIT either
    assert [c for c, _ in r.calls].count("SETBIT") == calls.count("SETBIT")
    big.driver.close()
    small = pkg.Bloomfilter(size=10000, error_rate=0.01, key_name="small", driver="hip", redis=pkg.FakeRedis())
    ks = ["s%d" % i for i in range(5000)]
    assert not small.driver._setbit_sync(pkg.keys.pack(ks)[1])
    small.insert_many(ks)
    assert "SETRANGE" in [c for c, _ in small.redis.calls]
    assert small.redis.get("small") == small.driver.to_redis_string()
    small.driver.close()
