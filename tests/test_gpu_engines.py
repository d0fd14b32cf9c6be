"""The RubyTest hash engines on the GPU (lib/bloomfilter_driver/ruby_test.rb:43-61).

Offsets against the committed golden vectors (hashlib restatement, cross-checked by Node's
crypto) and against ``oracle.py_engine_indexes``; inserts and include? against a
SETBIT/GETBIT model over those offsets; the ``hip-test`` driver against a restatement of
RubyTest over FakeRedis.
"""
import json
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def flags(pkg, engine):
    return pkg.BF_FLAG_ENGINE_MD5 if engine == "md5" else pkg.BF_FLAG_ENGINE_SHA1


def test_engine_indexes_match_golden(pkg):
    """Every golden regime whose bitset is small enough for a test (m <= 2^36 bits); the
    2^40 / 2^63 / 2^64 regimes pin the oracle only (test_engine_indexes_large_modulus
    covers the device's 128-bit reduction)."""
    with open(os.path.join(HERE, "golden", "golden.json")) as fh:
        vecs = json.load(fh)["engine_indexes"]
    groups = {}
    for v in vecs:
        groups.setdefault((v["engine"], int(v["m"]), v["k"]), []).append(v)
    tested = 0
    for (engine, m, k), vs in groups.items():
        if m > 2**36:
            continue
        buf, offs = pkg.keys.pack([bytes.fromhex(v["key_hex"]) for v in vs])
        with pkg.Filter(m, k, flags=flags(pkg, engine)) as f:
            got = f.indexes_many(buf, offs)
        want = np.array([[int(x) for x in v["idx"]] for v in vs], dtype=np.uint64)
        np.testing.assert_array_equal(got, want, err_msg="%s m=%d k=%d" % (engine, m, k))
        tested += 1
    assert tested == 8


@pytest.mark.parametrize("engine", ["md5", "sha1"])
def test_engine_indexes_large_modulus(pkg, engine):
    """m up to 2^37 bits (16 GiB of HBM): the 128/160-bit digest mod a 38-bit m."""
    rng = np.random.default_rng(81)
    keys = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in rng.integers(0, 130, 3000)]
    buf, offs = pkg.keys.pack(keys)
    for m, k in ((2**37 - 25, 13), (2**32 + 15, 64), (3, 5)):
        with pkg.Filter(m, k, flags=flags(pkg, engine)) as f:
            got = f.indexes_many(buf, offs)
        want = np.array([O.py_engine_indexes(kb, m, k, engine) for kb in keys], dtype=np.uint64)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("engine", ["md5", "sha1"])
@pytest.mark.parametrize("m,k,n", [(95851, 6, 5000), (9585058, 7, 40_000), (2**33 + 7, 13, 20_000)])
def test_engine_insert_include_match_setbit_model(pkg, engine, m, k, n):
    rng = np.random.default_rng(82)
    keys = ["e%d" % v for v in rng.integers(0, 10**9, n)]
    probe = keys[: n // 2] + ["x%d" % v for v in range(n // 2)]
    idx = np.array([O.py_engine_indexes(x, m, k, engine) for x in keys], dtype=np.uint64)
    model = np.zeros((m + 7) // 8, np.uint8)
    np.bitwise_or.at(model, (idx >> 3).astype(np.int64).ravel(),
                     (0x80 >> (idx & 7)).astype(np.uint8).ravel())
    nz = np.flatnonzero(model)
    want_s = model[: nz[-1] + 1].tobytes() if len(nz) else b""
    pidx = np.array([O.py_engine_indexes(x, m, k, engine) for x in probe], dtype=np.uint64)
    want_inc = ((model[(pidx >> 3).astype(np.int64)] & (0x80 >> (pidx & 7)).astype(np.uint8)) != 0).all(axis=1)
    with pkg.Filter(m, k, flags=flags(pkg, engine)) as f:
        buf, offs = pkg.keys.pack(keys)
        any1, _ = f.insert_many(buf, offs, any_new=True)
        any2, _ = f.insert_many(buf, offs, any_new=True)
        assert (any1, any2) == (True, False)
        assert f.export_redis() == want_s
        pb, po = pkg.keys.pack(probe)
        np.testing.assert_array_equal(f.include_many(pb, po).astype(bool), want_inc)
        with pytest.raises(pkg.ArgumentError):
            f.insert_many(buf, offs, per_key_new=True)


def test_engine_flags_refused_where_meaningless(pkg):
    with pytest.raises(pkg.ArgumentError):
        pkg.Filter(1000, 3, flags=pkg.BF_FLAG_ENGINE_MD5 | pkg.BF_FLAG_ENGINE_SHA1)
    with pytest.raises(pkg.ArgumentError):
        pkg.Filter(10**9, 3, shard_count=2, shard_index=0, flags=pkg.BF_FLAG_ENGINE_SHA1)


class RubyTestRestatement:
    """ruby_test.rb:17-68 over a redis-like client."""

    def __init__(self, options, redis):
        self.o, self.r = options, redis

    def insert(self, data, expire=None):
        changed = [self.r.setbit(self.o["key_name"], i, 1)
                   for i in O.py_engine_indexes(data, self.o["bits"], self.o["hashes"], self.o["hash_engine"])]
        if 0 in changed and expire:
            self.r.expire(self.o["key_name"], expire)

    def include(self, key):
        idx = O.py_engine_indexes(key, self.o["bits"], self.o["hashes"], self.o["hash_engine"])
        if self.r.getbit(self.o["key_name"], idx[0]) == 0:
            return False
        return all(self.r.getbit(self.o["key_name"], i) for i in idx[1:])


@pytest.mark.parametrize("engine", ["md5", "sha1"])
def test_hip_test_driver_matches_ruby_test(pkg, engine):
    r_hip, r_ref = pkg.FakeRedis(), pkg.FakeRedis()
    bf = pkg.Bloomfilter({"size": 10_000, "error_rate": 0.01, "key_name": "t", "redis": r_hip,
                          "driver": "hip-test", "hash_engine": engine})
    assert bf.options["hash_engine"] == engine and isinstance(bf.driver, pkg.HipTest)
    ref = RubyTestRestatement(bf.options, r_ref)
    keys = ["k%d" % i for i in range(3000)] + list(range(200))
    for chunk in (keys[:1], keys[1:1500], keys[1500:]):
        bf.insert_many(chunk, 60)
        for key in chunk:
            ref.insert(key, 60)
        assert r_hip.get("t") == r_ref.get("t")
    assert r_hip.ttl("t") > 0
    probe = keys[:500] + ["n%d" % i for i in range(2000)]
    assert bf.include_many(probe).tolist() == [ref.include(p) for p in probe]
    bf.clear()
    assert r_hip.get("t") is None and not bf.include("k1")


def test_hip_test_default_engine_and_broken_crc32(pkg):
    bf = pkg.Bloomfilter({"size": 100, "error_rate": 0.01, "key_name": "d", "driver": "hip-test",
                          "redis": pkg.FakeRedis()})
    assert bf.options["hash_engine"] == "md5"          # bloomfilter.rb:15
    bf.insert("x")
    assert bf.include("x")
    crc = pkg.Bloomfilter({"size": 100, "error_rate": 0.01, "key_name": "c", "driver": "hip-test",
                           "hash_engine": "crc32", "redis": pkg.FakeRedis()})
    with pytest.raises(pkg.ArgumentError):
        crc.insert("x")
    with pytest.raises(pkg.ArgumentError):
        crc.include("x")
    crc.clear()                                           # DEL still works (ruby_test.rb:34-36)
    bad = pkg.Bloomfilter({"size": 100, "error_rate": 0.01, "key_name": "b", "driver": "hip-test",
                           "hash_engine": "sha256", "redis": pkg.FakeRedis()})
    with pytest.raises(NameError):
        bad.insert("x")


@pytest.mark.parametrize("engine", ["md5", "sha1"])
def test_spec_error_rate_with_engine(pkg, engine):
    """spec/redis_bloomfilter_spec.rb:100-106's error-rate loop, RubyTest engines."""
    bf = pkg.Bloomfilter({"size": 100, "error_rate": 0.02, "key_name": "__test_bf", "driver": "hip-test",
                          "hash_engine": engine, "redis": pkg.FakeRedis()})
    rng = np.random.default_rng(83)
    visited, errors = set(), 0
    for _ in range(180):
        a = int(rng.integers(0, 180))
        errors += bf.include(a) != (a in visited)
        visited.add(a)
        bf.insert(a)
    assert round(errors / 180, 2) <= 0.02
