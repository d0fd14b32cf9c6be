"""Incremental Redis sync: the dirty-block map of ``bf_track_dirty``.

What the hip driver writes back after an insert must rebuild exactly the string the
SETBIT path would leave in Redis (ruby.rb:57-63), while sending only the 64 KiB blocks
the batch could have changed.  For every insert path (direct, binned, sequential
per-key flags) the reported blocks are checked against the oracle's offsets:

    blocks whose bytes changed  ⊆  reported blocks  ⊆  blocks some probe of the batch hit
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BLOCK = 65536


def rand_keys(rng, n, lo=0, hi=40):
    lens = rng.integers(lo, hi + 1, size=n)
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    return rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8), offs


def padded(s: bytes, size: int) -> np.ndarray:
    a = np.zeros(size, np.uint8)
    a[: len(s)] = np.frombuffer(s, np.uint8)
    return a


def blocks_of(ranges):
    out = set()
    for off, n in ranges:
        assert off % BLOCK == 0 and n > 0
        out.update(range(off // BLOCK, (off + n - 1) // BLOCK + 1))
    return out


@pytest.mark.parametrize("path", ["direct", "binned", "seq"])
@pytest.mark.parametrize("m,k,n", [(1437758757, 10, 300), (1437758757, 10, 200_000), (9585058, 6, 50_000)])
def test_dirty_blocks_bound_the_change(pkg, oracle, monkeypatch, path, m, k, n):
    monkeypatch.setenv("BFHIP_INSERT_BINNED", "1" if path == "binned" else "0")
    rng = np.random.default_rng(71)
    first, second = rand_keys(rng, 150_000), rand_keys(rng, n)
    with pkg.Filter(m, k) as f:
        f.insert_many(*first)                       # before tracking: not reported
        f.track_dirty(True)
        assert f.dirty_ranges() == ([], f.redis_len())
        s0 = f.export_redis()
        f.insert_many(*second, per_key_new=(path == "seq"))
        s1 = f.export_redis()
        ranges, rlen = f.dirty_ranges(clear=True)
        assert rlen == len(s1)
        assert all(off + ln <= rlen for off, ln in ranges)
        size = max(len(s0), len(s1))
        a0, a1 = padded(s0, size), padded(s1, size)
        diff = np.flatnonzero(a0 != a1)
        changed = set((diff // BLOCK).tolist())
        idx = oracle.indexes_many(second[0], second[1], m, k).reshape(-1)
        touched = set(np.unique(idx >> 19).tolist())
        got = blocks_of(ranges)
        assert changed <= got <= touched
        # replaying the ranges onto the old string gives the new one, as the driver does
        r = pkg.FakeRedis()
        if s0:
            r.set("bf", s0)
        for off, ln in ranges:
            r.setrange("bf", off, f.export_range(off, ln))
        assert (r.get("bf") or b"") == s1
        assert f.dirty_ranges() == ([], rlen)     # cleared
        f.insert_many(*second)                    # nothing new -> nothing dirty
        assert f.dirty_ranges()[0] == []


def test_import_clear_and_bounds(pkg):
    m, k = 9585058, 6
    with pkg.Filter(m, k) as f:
        with pytest.raises(pkg.ArgumentError):
            f.dirty_ranges()                      # tracking off
        f.track_dirty(True)
        assert f.dirty_ranges() == ([], 0)
        f.import_redis(b"\x00" * 10 + b"\x01", pkg.BF_IMPORT_OR)
        ranges, rlen = f.dirty_ranges()
        assert rlen == 11 and ranges == [(0, 11)]  # everything clipped to the trimmed string
        f.insert_many(*pkg.keys.pack(["a", "b"]))
        f.clear()
        assert f.dirty_ranges() == ([], 0)
        with pytest.raises(pkg.ArgumentError):
            f.export_range(f.device_bytes - 4, 8)
        assert f.export_range(0, 0) == b""
        f.track_dirty(False)
        with pytest.raises(pkg.ArgumentError):
            f.dirty_ranges()


def test_driver_write_through_sends_only_changed_blocks(pkg, oracle):
    """hip driver on a ~120 MB filter: after every batch the Redis key equals the device string
    (= the SETBIT result), and the bytes sent are bounded by the blocks the batch touched."""
    r = pkg.FakeRedis()
    bf = pkg.Bloomfilter({"size": 100_000_000, "error_rate": 0.01, "key_name": "big", "redis": r,
                          "driver": "hip"})
    m, k = bf.options["bits"], bf.options["hashes"]
    rng = np.random.default_rng(72)
    for n in (1, 1, 10, 1000, 100_000):
        batch = ["k%d" % v for v in rng.integers(0, 10**12, n)]
        before = r.bytes_in
        bf.insert_many(batch)
        assert r.get("big") == bf.driver.to_redis_string()
        buf, offs = pkg.keys.pack(batch)
        touched = np.unique(oracle.indexes_many(buf, offs, m, k).reshape(-1) >> 19)
        assert r.bytes_in - before <= len(touched) * BLOCK
        if n == 10:   # 12 keys so far: a few MB at most of a ~120 MB string
            assert r.bytes_in <= 12 * k * BLOCK < len(r.get("big")) / 10
    # a second driver attached to the same key starts clean: its first insert sends blocks only
    other = pkg.Bloomfilter({"size": 100_000_000, "error_rate": 0.01, "key_name": "big", "redis": r,
                             "driver": "hip"})
    before = r.bytes_in
    other.insert("fresh-key")
    assert r.bytes_in - before <= k * BLOCK
    assert r.get("big") == other.driver.to_redis_string()
    assert bf.driver.flush() == 0                 # bf's own changes were all written already
    bf.clear()
    assert r.get("big") is None


def test_chunked_sync_beyond_512mb(pkg):
    """A 750 MB filter through a server whose proto-max-bulk-len admits it: writes go out as
    SETRANGE calls of <= chunk_bytes, a new driver reads the key back with GETRANGE chunks;
    stock Redis (512 MB cap) refuses the string as it would refuse the SETBITs."""
    chunk = 64 << 20
    r = pkg.FakeRedis(max_string=1 << 30)
    opts = {"size": 626_000_000, "error_rate": 0.01, "key_name": "huge", "redis": r, "driver": "hip",
            "chunk_bytes": chunk}
    bf = pkg.Bloomfilter(dict(opts))
    keys = np.arange(1 << 20, dtype=np.int64) * 7919
    r.calls.clear()
    bf.insert_many(keys)
    s = bf.driver.to_redis_string()
    assert len(s) > 600 << 20
    n_set = sum(1 for c, _ in r.calls if c == "SETRANGE")
    assert n_set >= len(s) // chunk and r.get("huge") == s
    other = pkg.Bloomfilter(dict(opts))                    # attach: GETRANGE chunks
    assert sum(1 for c, _ in r.calls if c == "GETRANGE") >= len(s) // chunk
    assert other.driver.to_redis_string() == s
    assert other.include_many(keys[:5000]).all()
    stock = pkg.FakeRedis()
    small = pkg.Bloomfilter(dict(opts, redis=stock, key_name="huge2"))
    with pytest.raises(pkg.fakeredis.ResponseError):
        small.insert_many(keys)


def test_manual_sync_flushes_changes_since_last_flush(pkg):
    r = pkg.FakeRedis()
    bf = pkg.Bloomfilter({"size": 10_000_000, "error_rate": 0.01, "key_name": "man", "redis": r,
                          "driver": "hip", "sync": "manual"})
    bf.insert_many(["a%d" % i for i in range(50_000)])
    assert r.get("man") is None
    sent = bf.driver.flush()
    assert r.get("man") == bf.driver.to_redis_string() and 0 < sent <= len(r.get("man"))
    assert bf.driver.flush() == 0
    bf.insert("one-more")
    assert 0 < bf.driver.flush() <= bf.options["hashes"] * BLOCK
    assert r.get("man") == bf.driver.to_redis_string()
    assert bf.driver.flush(full=True) == len(r.get("man"))
