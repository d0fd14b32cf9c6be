"""Host logic of the Redis::Bloomfilter mirror (CPU only): option validation,
sizing, driver resolution, key marshalling and the Redis string model.

Mirrors spec/redis_bloomfilter_spec.rb:28-60 (the mocked, Redis-free cases).
"""
import numpy as np
import pytest


class FakeRubyDriver:
    def __init__(self, options):
        self.options = options
        self.redis = None


class FakeLuaDriver(FakeRubyDriver):
    pass


@pytest.fixture
def registry(pkg):
    saved = dict(pkg.DRIVERS)
    pkg.register_driver(FakeRubyDriver, "Ruby")
    pkg.register_driver(FakeLuaDriver, "Lua")
    yield pkg.DRIVERS
    pkg.DRIVERS.clear()
    pkg.DRIVERS.update(saved)


def test_version(pkg):   # spec:28-30
    assert pkg.Bloomfilter.version() == "redis-bloomfilter version %s" % pkg.Bloomfilter.VERSION


def test_initialize_options(pkg, registry):   # spec:32-37
    with pytest.raises(pkg.ArgumentError):
        pkg.Bloomfilter()
    with pytest.raises(pkg.ArgumentError):
        pkg.Bloomfilter(size=123)
    with pytest.raises(pkg.ArgumentError):
        pkg.Bloomfilter(error_rate=0.01)
    with pytest.raises(NameError):
        pkg.Bloomfilter(size=123, error_rate=0.01, driver="bibu")


def test_driver_by_redis_version(pkg, registry):   # spec:39-50
    r26 = pkg.FakeRedis(version="2.6.0")
    r25 = pkg.FakeRedis(version="2.5.0")
    bf = pkg.Bloomfilter(size=1000, error_rate=0.01, key_name="ossom", redis=r26)
    assert isinstance(bf.driver, FakeLuaDriver)
    bf = pkg.Bloomfilter(size=1000, error_rate=0.01, key_name="ossom", redis=r25)
    assert type(bf.driver) is FakeRubyDriver
    assert bf.driver.redis is r25


def test_options_computed(pkg, registry):   # spec:52-60 (sizing part)
    bf = pkg.Bloomfilter(size=1000, error_rate=0.01, key_name="ossom", driver="ruby")
    assert bf.options["size"] == 1000
    assert bf.options["bits"] == 9585
    assert bf.options["hashes"] == 6
    assert bf.options["key_name"] == "ossom"
    assert bf.driver.options["bits"] == 9585     # the driver receives the whole hash (bloomfilter.rb:44)


def test_driver_name(pkg):   # bloomfilter.rb:77-79
    assert pkg.driver_name("ruby-test") == "RubyTest"
    assert pkg.driver_name("hip") == "Hip"
    assert pkg.driver_name("LUA") == "Lua"
    assert pkg.driver_name("ruby_test") == "Ruby_test"
    assert "Hip" in pkg.DRIVERS


def test_optimal_m_k_edge_semantics(pkg):
    B = pkg.Bloomfilter
    assert B.optimal_m(1000, 0.01) == 9585
    assert B.optimal_k(1000, 9585) == 6
    assert B.optimal_k(1000.0, 9585) == 7           # Float size: 9.585 * ln2 = 6.64 -> 7 (no floor)
    assert B.optimal_k(10, 3) == 1                  # 0 bumped to 1
    with pytest.raises(ZeroDivisionError):
        B.optimal_k(0, 0)
    with pytest.raises(FloatingPointError):         # Ruby: FloatDomainError (Infinity.round)
        B.optimal_m(100, 0.0)


def test_key_to_s(pkg):
    to_s = pkg.keys.to_s
    assert to_s("asdlol") == b"asdlol"
    assert to_s(42) == b"42" and to_s(-7) == b"-7" and to_s(np.int64(5)) == b"5"
    assert to_s(None) == b"" and to_s(True) == b"true" and to_s(False) == b"false"
    assert to_s(1.0) == b"1.0" and to_s(1e16) == b"1.0e+16" and to_s(1e-5) == b"1.0e-05"
    assert to_s(1e15) == b"1000000000000000.0" and to_s(0.0001) == b"0.0001"
    assert to_s("é") == "é".encode()
    with pytest.raises(TypeError):
        to_s(object())


def test_pack_and_pack_decimal(pkg):
    buf, offs = pkg.keys.pack(["a", "", "bcd", 12])
    assert offs.tolist() == [0, 1, 1, 4, 6]
    assert bytes(buf) == b"abcd12"
    vals = np.array([0, 9, 10, 99, 100, -1, -12345, 2**63 - 1, -2**63], dtype=np.int64)
    b, o = pkg.keys.pack_decimal(vals)
    assert [pkg.keys.unpack(b, o, i) for i in range(len(vals))] == [str(int(v)).encode() for v in vals]
    b, o = pkg.keys.pack(np.arange(1000, dtype=np.uint32))
    assert pkg.keys.unpack(b, o, 999) == b"999"
    b, o = pkg.keys.pack([])
    assert len(b) == 0 and o.tolist() == [0]


def test_fakeredis_bit_semantics(pkg):
    r = pkg.FakeRedis()
    assert r.getbit("k", 100) == 0
    assert r.setbit("k", 7, 1) == 0
    assert r.get("k") == b"\x01"
    assert r.setbit("k", 0, 1) == 0
    assert r.get("k") == b"\x81"
    assert r.setbit("k", 0, 1) == 1
    assert r.setbit("k", 17, 1) == 0
    assert r.get("k") == b"\x81\x00\x40"       # grows to offset/8 + 1, MSB-first
    assert r.getbit("k", 17) == 1 and r.getbit("k", 16) == 0 and r.getbit("k", 10**6) == 0
    assert r.setrange("k", 5, b"\xff") == 6
    assert r.get("k") == b"\x81\x00\x40\x00\x00\xff"
    assert r.getrange("k", 0, 1) == b"\x81\x00" and r.getrange("k", -1, -1) == b"\xff"
    with pytest.raises(pkg.fakeredis.ResponseError):
        r.setbit("k", 2**32, 1)


def test_fakeredis_ttl(pkg):
    now = [0.0]
    r = pkg.FakeRedis(clock=lambda: now[0])
    r.setbit("k", 3, 1)
    assert r.ttl("k") == -1 and r.ttl("missing") == -2
    assert r.expire("k", 120) is True
    assert r.ttl("k") == 120
    r.setrange("k", 0, b"\x10")               # SETRANGE keeps the TTL
    assert r.ttl("k") == 120
    now[0] = 119.5
    assert r.exists("k") == 1
    now[0] = 120.0
    assert r.get("k") is None and r.ttl("k") == -2
    r.set("j", b"x")
    r.expire("j", 5)
    r.set("j", b"y")                          # SET clears it
    assert r.ttl("j") == -1
    assert r.delete("j", "nope") == 1
    assert r.keys("*") == []


def test_replicated_merge_gathered(pkg):
    """distributed.merge_gathered: the all-gathered batches minus this rank's, as one packed
    batch whose keys are exactly the other ranks' keys in rank order (CPU tensors)."""
    import torch
    D = pkg.distributed
    batches = [["a", "bb", ""], [], ["ccc", "d" * 300], ["x"]]
    max_b = max(max(sum(len(k) for k in b) for b in batches), 1)
    max_n = max(len(b) for b in batches)
    gk = torch.zeros(len(batches) * max_b, dtype=torch.uint8)
    gl = torch.zeros(len(batches) * max_n, dtype=torch.int32)
    sizes = []
    for r, b in enumerate(batches):
        raw = "".join(b).encode()
        gk[r * max_b: r * max_b + len(raw)] = torch.tensor(list(raw), dtype=torch.uint8)
        gl[r * max_n: r * max_n + len(b)] = torch.tensor([len(k) for k in b], dtype=torch.int32)
        sizes.append((len(raw), len(b), max([len(k) for k in b], default=0)))
    for skip in range(len(batches)):
        kb, ko, n = D.merge_gathered(gk, gl, sizes, max_b, max_n, skip)
        want = [k for r, b in enumerate(batches) if r != skip for k in b]
        assert n == len(want)
        o = ko.tolist()
        got = [bytes(kb[o[j]: o[j + 1]].tolist()).decode() for j in range(n)]
        assert got == want
        assert kb.numel() == o[-1] + 16


class RecordingDriver(FakeRubyDriver):
    def insert(self, data, expire):
        self.last_expire = expire


def test_expire_keeps_ruby_truthiness(pkg, registry):
    """bloomfilter.rb:62 `expire || @options[:default_expire]`: nil and false take the default,
    0 is truthy in Ruby and is passed on (ruby.rb:62 then EXPIREs with 0, deleting the key)."""
    pkg.register_driver(RecordingDriver, "Recording")
    bf = pkg.Bloomfilter(size=100, error_rate=0.01, driver="recording", default_expire=60)
    for given, want in [(None, 60), (False, 60), (0, 0), (5, 5)]:
        bf.insert("x", given)
        assert bf.driver.last_expire == want, given


def test_fakeredis_pttl_and_expire_zero(pkg):
    now = [0.0]
    r = pkg.FakeRedis(clock=lambda: now[0])
    r.setbit("k", 3, 1)
    assert r.pttl("k") == -1 and r.pttl("missing") == -2
    r.expire("k", 2)
    now[0] = 0.25
    assert r.pttl("k") == 1750 and r.ttl("k") == 2
    assert r.expire("k", 0) is True and r.exists("k") == 0   # EXPIRE 0 deletes, like Redis


def test_oracle_restatements_expire_zero(pkg, O):
    """The ruby.rb / add.lua restatements EXPIRE on 0 (Ruby and Lua truthiness)."""
    import lua_oracle
    r = pkg.FakeRedis()
    ruby = O.RubyDriverRestatement({"bits": 9585, "hashes": 6, "key_name": "bf", "redis": r})
    ruby.insert("asdlol", 0)
    assert r.exists("bf") == 0 and ruby.include("asdlol") is False
    ruby.insert("asdlol")
    assert r.exists("bf") == 1 and r.ttl("bf") == -1 and ruby.include("asdlol") is True
    lua_oracle.add(r, "lb", 1000, 0.01, "asdlol", 0)
    assert r.exists("lb:1") == 0 and r.get("lb:count") == b"1"
    assert lua_oracle.check(r, "lb", 1000, 0.01, "asdlol") is False
