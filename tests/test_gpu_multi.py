"""Multi-device handles (bf_config.device_count / devices / mode, bf_multi.cpp) through the
C ABI, against the oracle.  The box has one GPU, so a device may repeat: devices = [0, 0, 0]
is three shard (or replica) handles on GPU 0, whose windows still travel by
hipMemcpyPeerAsync — the same code path as three GPUs over xGMI.  devices = [0] is the
cfg form the Ruby driver's `devices:` option sends (lib/redis/bloomfilter.rb:43-45)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED + 40


def _roundtrip(pkg, oracle, m, k, devices, mode, n=60_000, **fkw):
    rng = np.random.default_rng(SEED + len(devices))
    ib, io = pkg.keys.pack_decimal(rng.integers(0, 10**12, size=n))
    pb, po = pkg.keys.pack_decimal(rng.integers(0, 10**12, size=n // 2))
    probe = (np.concatenate([ib, pb]), np.concatenate([io, po[1:] + io[-1]]))
    bits = oracle.new_bitset(m, k)
    oracle.insert_many(bits, m, k, ib, io)
    want = oracle.redis_string(bits)
    want_inc = oracle.include_many(bits, m, k, *probe)
    with pkg.Filter(m, k, devices=devices, mode=mode, **fkw) as f:
        assert f.reach_bits == min(m, k * 0xFFFFFFFF + 1)
        any1, _ = f.insert_many(ib, io, any_new=True)
        any2, _ = f.insert_many(ib, io, any_new=True)
        assert (any1, any2) == (True, False)
        got = f.export_redis()
        assert f.redis_len() == len(want)
        assert hashlib.sha1(got).hexdigest() == hashlib.sha1(want).hexdigest()
        np.testing.assert_array_equal(f.include_many(*probe), want_inc)
        # a byte range straddling ownership blocks
        if len(want) > 300_000:
            assert f.export_range(131_000, 150_000) == want[131_000:281_000]
        np.testing.assert_array_equal(f.indexes_many(ib, io[:9]), oracle.indexes_many(ib, io[:9], m, k))
        # import (replace) into a cleared filter, then OR a second string in
        f.clear()
        assert f.export_redis() == b""
        f.import_redis(want)
        assert f.export_redis() == want
        jb, jo = pkg.keys.pack(["x%d" % i for i in range(5000)])
        bits2 = oracle.new_bitset(m, k)
        oracle.insert_many(bits2, m, k, jb, jo)
        f.import_redis(oracle.redis_string(bits2), mode=1)
        assert f.export_redis() == oracle.redis_string(np.bitwise_or(bits, bits2))
    return want


@pytest.mark.parametrize("mode", ["replicated", "partitioned"])
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_matches_oracle(pkg, oracle, devices, mode):
    _roundtrip(pkg, oracle, 9585058, 6, devices, mode)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0]])
def test_partitioned_past_2_32_bits_per_shard(pkg, oracle, devices):
    """The north-star filter (1.2 GB) over 2 shards: 4.8e9 bits each, so every owner takes
    two 2^32-bit sub-range windows (nh = 2); over 4 shards one (nh = 1)."""
    _roundtrip(pkg, oracle, 9585058377, 6, devices, "partitioned", n=40_000, shard_block_log2=20)


def test_partitioned_small_blocks_and_chunks(pkg, oracle):
    """Small ownership blocks (2^10 bits) and a batch split into many rounds."""
    _roundtrip(pkg, oracle, 95851, 7, [0, 0, 0], "partitioned", n=20_000, shard_block_log2=10)


def test_multi_device_flags_and_dirty(pkg, oracle):
    m, k = 1437758757, 10
    rng = np.random.default_rng(SEED)
    b, o = pkg.keys.pack_decimal(rng.integers(0, 3000, size=5000))   # repeats: sequential flags differ
    bits = oracle.new_bitset(m, k)
    want_any, want_pk = oracle.insert_many(bits, m, k, b, o, per_key=True)
    with pkg.Filter(m, k, devices=[0, 0], mode="replicated") as f:
        any_new, pk = f.insert_many(b, o, any_new=True, per_key_new=True)
        np.testing.assert_array_equal(pk, want_pk)
        assert any_new == bool(want_any)
    with pkg.Filter(m, k, devices=[0, 0, 0], mode="partitioned") as f:
        with pytest.raises(pkg.ArgumentError, match="per_key_new"):
            f.insert_many(b, o, per_key_new=True)
        # dirty ranges of a partitioned handle: replaying them rebuilds the string exactly
        f.track_dirty(True)
        f.insert_many(b, o)
        ranges, rlen = f.dirty_ranges(clear=True)
        want = oracle.redis_string(bits)
        assert rlen == len(want)
        rebuilt = bytearray(rlen)
        for off, ln in ranges:
            rebuilt[off: off + ln] = f.export_range(off, ln)
        assert bytes(rebuilt) == want
        assert sum(ln for _, ln in ranges) < rlen   # only the touched blocks
        assert f.dirty_ranges(clear=True)[0] == []


def test_multi_device_refuses_device_api(pkg):
    with pkg.Filter(95851, 6, devices=[0, 0], mode="partitioned") as f:
        with pytest.raises(pkg.ArgumentError, match="multi-device"):
            f.device_bits()
    with pytest.raises(pkg.ArgumentError):
        pkg.Filter(95851, 6, devices=[0, 99], mode="replicated")


def test_hip_driver_devices_option(pkg, oracle):
    """Redis::Bloomfilter.new(driver: 'hip', devices: [...], mode: ...) — the facade passes its
    whole options hash to the driver (bloomfilter.rb:44), as the Ruby driver's cfg does."""
    r = pkg.FakeRedis()
    for mode in ("replicated", "partitioned"):
        bf = pkg.Bloomfilter({"size": 10_000, "error_rate": 0.01, "key_name": "bf_" + mode, "redis": r,
                              "driver": "hip", "devices": [0, 0], "mode": mode})
        keys = ["k%d" % i for i in range(3000)]
        bf.insert_many(keys)
        assert bf.include_many(keys).all()
        ref = pkg.FakeRedis()
        import oracle as O
        rd = O.RubyDriverRestatement({"bits": bf.options["bits"], "hashes": bf.options["hashes"], "key_name": "x",
                                      "redis": ref})
        for key in keys:
            rd.insert(key)
        assert r.get("bf_" + mode) == ref.get("x")


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_partitioned_first_call_fewer_keys_than_devices(pkg, oracle, devices):
    """a fresh partitioned handle whose FIRST call is a one-key insert asking for
    any_new (the hip driver's per-key insert under write-through) — device slots with an
    empty part own windows too, so their flag and counts must exist before the owner loop.
    Then one- and two-key include?s, whose answer windows live on the requester's device."""
    m, k = 95851, 6
    for keys in (["solo"], ["a", "b"]):
        ib, io = pkg.keys.pack(keys)
        bits = oracle.new_bitset(m, k)
        oracle.insert_many(bits, m, k, ib, io)
        with pkg.Filter(m, k, devices=devices, mode="partitioned") as f:
            any1, _ = f.insert_many(ib, io, any_new=True)
            any2, _ = f.insert_many(ib, io, any_new=True)
            assert (any1, any2) == (True, False)
            assert f.export_redis() == oracle.redis_string(bits)
            pb, po = pkg.keys.pack(keys[:1])
            assert f.include_many(pb, po).tolist() == [1]
            qb, qo = pkg.keys.pack(keys + ["absent-%d" % i for i in range(3)])
            np.testing.assert_array_equal(f.include_many(qb, qo), oracle.include_many(bits, m, k, qb, qo))
