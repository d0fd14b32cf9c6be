"""The ``hip`` driver behind the facade, against the reference spec's cases
(spec/redis_bloomfilter_spec.rb:52-60, 89-120) with FakeRedis standing in for
redis-server, plus interop with the ruby driver's Redis string.
"""
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def factory(pkg, options, driver="hip", **kw):   # spec:19-22
    options = dict(options)
    options["driver"] = driver
    options.update(kw)
    return pkg.Bloomfilter(options)


def error_rate(bf, elems, rng):   # spec:7-17
    visited = set()
    error = 0
    for _ in range(elems):
        a = rng.randrange(elems)
        if bf.include(a) != (a in visited):
            error += 1
        visited.add(a)
        bf.insert(a)
    return error / elems


def test_create(pkg):   # spec:52-60
    r = pkg.FakeRedis()
    bf = factory(pkg, {"size": 1000, "error_rate": 0.01, "key_name": "ossom", "redis": r})
    assert bf.options["size"] == 1000
    assert bf.options["bits"] == 9585
    assert bf.options["hashes"] == 6
    assert bf.options["key_name"] == "ossom"
    assert isinstance(bf.driver, pkg.Hip)
    bf.clear()


def test_should_work(pkg):   # spec:90-98
    r = pkg.FakeRedis()
    bf = factory(pkg, {"size": 1000, "error_rate": 0.01, "key_name": "__test_bf", "redis": r})
    bf.clear()
    assert bf.include("asdlol") is False
    bf.insert("asdlol")
    assert bf.include("asdlol") is True
    bf.clear()
    assert bf.include("asdlol") is False
    assert r.get("__test_bf") is None


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_honor_error_rate(pkg, seed):   # spec:100-106
    bf = factory(pkg, {"size": 100, "error_rate": 0.02, "key_name": "__test_bf", "redis": pkg.FakeRedis()})
    bf.clear()
    e = error_rate(bf, 180, random.Random(seed))
    assert round(e, 2) <= round(bf.options["error_rate"], 2)


def test_add_element(pkg):   # spec:108-112
    bf = factory(pkg, {"size": 100, "error_rate": 0.01, "key_name": "__test_bf", "redis": pkg.FakeRedis()})
    bf.insert("asdlolol")
    assert bf.include("asdlolol") is True


def test_ttl(pkg):   # spec:114-118 (+ README expiry semantics)
    now = [1000.0]
    r = pkg.FakeRedis(clock=lambda: now[0])
    bf = factory(pkg, {"size": 100, "error_rate": 0.01, "key_name": "__test_bf_hip", "redis": r,
                       "clock": lambda: now[0]})
    bf.insert("asdlolol", 120)
    assert r.ttl("__test_bf_hip") > 0
    bf.insert("other")                      # no expire given: TTL untouched (SETRANGE keeps it)
    assert r.ttl("__test_bf_hip") == 120
    now[0] += 121                           # key expired in Redis -> device copy follows
    assert bf.include("asdlolol") is False
    assert r.get("__test_bf_hip") is None


def test_default_expire(pkg):
    r = pkg.FakeRedis()
    bf = factory(pkg, {"size": 100, "error_rate": 0.01, "key_name": "k", "redis": r, "default_expire": 60})
    bf.insert("x")
    assert 0 < r.ttl("k") <= 60


def test_expire_only_when_new(pkg):
    """ruby.rb:61-62: EXPIRE only when some bit flipped."""
    r = pkg.FakeRedis()
    bf = factory(pkg, {"size": 100, "error_rate": 0.01, "key_name": "k", "redis": r})
    bf.insert("x")
    r.calls.clear()
    bf.insert("x", 30)
    assert ("EXPIRE", "k") not in r.calls
    assert r.ttl("k") == -1


def test_write_through_string_equals_ruby_driver(pkg, O):
    """Same insert sequence -> byte-identical Redis string as the ruby driver (SETBIT path)."""
    r_hip, r_ruby = pkg.FakeRedis(), pkg.FakeRedis()
    bf = factory(pkg, {"size": 10_000, "error_rate": 0.01, "key_name": "bf", "redis": r_hip})
    ruby = O.RubyDriverRestatement({"bits": bf.options["bits"], "hashes": bf.options["hashes"],
                                    "key_name": "bf", "redis": r_ruby})
    keys = ["w%dq" % i for i in range(3000)] + list(range(500))
    for chunk in (keys[:1], keys[1:1000], keys[1000:]):
        bf.insert_many(chunk)
        for key in chunk:
            ruby.insert(key)
        assert r_hip.get("bf") == r_ruby.get("bf")
    assert len(r_hip.get("bf")) == len(r_ruby.get("bf"))


def test_reads_filter_written_by_ruby_driver(pkg, O):
    r = pkg.FakeRedis()
    m, k = pkg.Bloomfilter.optimal_m(10_000, 0.01), 6
    ruby = O.RubyDriverRestatement({"bits": m, "hashes": k, "key_name": "shared", "redis": r})
    members = ["m%d" % i for i in range(2000)]
    for key in members:
        ruby.insert(key)
    r.expire("shared", 500)
    bf = factory(pkg, {"size": 10_000, "error_rate": 0.01, "key_name": "shared", "redis": r})
    probe = members + ["x%d" % i for i in range(2000)]
    got = bf.include_many(probe)
    want = [ruby.include(p) for p in probe]
    assert got.tolist() == want
    assert got[:2000].all()
    # and the ruby driver reads what the hip driver adds
    bf.insert_many(["late%d" % i for i in range(100)])
    assert all(ruby.include("late%d" % i) for i in range(100))
    assert r.ttl("shared") > 0           # SETRANGE write-back kept the TTL


def test_manual_sync(pkg, O):
    r = pkg.FakeRedis()
    bf = factory(pkg, {"size": 10_000, "error_rate": 0.01, "key_name": "man", "redis": r, "sync": "manual"})
    bf.insert_many([str(i) for i in range(100)])
    assert r.get("man") is None
    n = bf.driver.flush()
    assert r.get("man") is not None and len(r.get("man")) == n
    bf.clear()
    assert r.get("man") is None


def test_batched_api_matches_single(pkg):
    r = pkg.FakeRedis()
    bf = factory(pkg, {"size": 50_000, "error_rate": 0.001, "key_name": "b", "redis": r, "sync": "manual"})
    keys = np.arange(20_000, dtype=np.int64)
    bf.insert_many(keys[:10_000])
    inc = bf.include_many(keys)
    assert inc[:10_000].all()
    assert inc[10_000:].mean() < 0.01
    assert [bf.include(int(x)) for x in keys[9990:10010]] == inc[9990:10010].tolist()


def test_lua_driver_name_is_not_registered(pkg):
    """spec:122-128's scalable layout runs on the GPU as driver 'hip-lua' (tests/test_gpu_lua.py);
    'lua' (the EVALSHA driver, lua.rb) stays the reference's own and resolves to nothing here."""
    with pytest.raises(NameError):
        factory(pkg, {"size": 100, "error_rate": 0.02, "key_name": "x"}, driver="lua")
