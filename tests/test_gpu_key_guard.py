"""Inconsistent key offsets on the device entry points.

ruby.rb:42 hashes `data.to_s`: every key has a finite length.  The *_dev entry points take
device offsets they cannot read without a sync, so every hashing kernel checks each key
against its tile's first and last offsets (bfdev::key_ok, the rule bf_check_offsets applies)
and hashes a key that fails as the empty string.  The handle's key-status word then makes
the next call (here bf_sync) return BF_EINVAL once.  Round 5's hang was a key end read back
as 0 (a wrapped length: ~2^26 SHA-1 blocks in one lane); here that case returns in
milliseconds with an error instead.
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def batch(n, seed=0x5EED):
    keys = [("key-%d-%d" % (seed, i)).encode() for i in range(n)]
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum([len(x) for x in keys], out=offs[1:])
    buf = np.frombuffer(b"".join(keys) + b"\0" * 16, np.uint8).copy()
    return keys, buf, offs


def dev(buf, offs):
    return torch.from_numpy(buf).cuda(), torch.from_numpy(offs.view(np.int64).copy()).cuda()


def empty_words():
    d = hashlib.sha1(b"").digest()
    return np.frombuffer(d[:16], ">u4").astype(np.uint32)


def expect_einval_once(pkg, f):
    torch.cuda.synchronize()
    with pytest.raises(pkg.ArgumentError, match="key offsets were inconsistent"):
        f.sync()
    f.sync()   # reported once


def test_good_offsets_raise_nothing(pkg):
    _, buf, offs = batch(3000)
    dk, do = dev(buf, offs)
    with pkg.Filter(9585058, 6) as f:
        out = torch.empty(3000, dtype=torch.uint8, device="cuda")
        f.insert_many_dev(dk.data_ptr(), do.data_ptr(), 3000)
        f.include_many_dev(dk.data_ptr(), do.data_ptr(), 3000, out.data_ptr())
        torch.cuda.synchronize()
        f.sync()
        assert out.cpu().numpy().all()


@pytest.mark.parametrize("case", ["backwards", "wrapped_end", "huge_last"])
def test_include_many_dev_bad_offsets_einval(pkg, oracle, case):
    n = 3000
    keys, buf, offs = batch(n)
    bad = offs.copy()
    if case == "backwards":        # key 1000 ends before it starts
        bad[1001] = bad[1000] - 3
    elif case == "wrapped_end":    # the r05 hang: a key end read back as 0 (the batch's last offset)
        bad[n] = 0
    else:                          # a last offset far past the buffer: key n-1 would be 2^40 bytes long
        bad[n] = np.uint64(1) << np.uint64(40)
    m, k = 9585058, 6
    dk, do = dev(buf, offs)
    _, dbo = dev(buf, bad)
    with pkg.Filter(m, k) as f:
        f.insert_many_dev(dk.data_ptr(), do.data_ptr(), n)
        torch.cuda.synchronize()
        f.sync()
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        f.include_many_dev(dk.data_ptr(), dbo.data_ptr(), n, out.data_ptr())   # returns: the kernel is async
        expect_einval_once(pkg, f)
        got = out.cpu().numpy()
        # keys of the tiles (256 keys) without a bad offset are answered as always
        tile = 1000 // 256 if case == "backwards" else (n - 1) // 256
        mask = np.ones(n, bool)
        mask[tile * 256:(tile + 1) * 256] = False
        assert got[mask].all()


def test_hash_many_dev_bad_key_is_the_empty_key(pkg):
    n = 600
    _, buf, offs = batch(n, seed=7)
    bad = offs.copy()
    bad[301] = bad[300] - 1          # key 300 runs backwards
    dk, dbo = dev(buf, bad)
    with pkg.Filter(9585058, 6) as f:
        dig = torch.empty((n, 4), dtype=torch.int32, device="cuda")
        f.hash_many_dev(dk.data_ptr(), dbo.data_ptr(), n, dig.data_ptr())
        expect_einval_once(pkg, f)
        words = dig.cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(words[300], empty_words())
        # a key of another tile is hashed as always
        want = np.frombuffer(hashlib.sha1(buf[int(offs[10]):int(offs[11])].tobytes()).digest()[:16], ">u4")
        np.testing.assert_array_equal(words[10], want.astype(np.uint32))


@pytest.mark.parametrize("binned", ["0", "1"])
def test_insert_many_dev_bad_offsets_einval(pkg, monkeypatch, binned):
    monkeypatch.setenv("BFHIP_INSERT_BINNED", binned)   # the direct kernel and the binned front (bin_front)
    n = 40_000
    _, buf, offs = batch(n, seed=11)
    bad = offs.copy()
    bad[20_001] = bad[20_000] - 5
    dk, dbo = dev(buf, bad)
    with pkg.Filter(9585058, 6) as f:
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        f.insert_many_dev(dk.data_ptr(), dbo.data_ptr(), n, flag.data_ptr())
        expect_einval_once(pkg, f)


def test_include_hash_dev_bad_next_offsets_einval(pkg):
    n = 2000
    _, buf, offs = batch(n, seed=3)
    _, nbuf, noffs = batch(n, seed=4)
    nbad = noffs.copy()
    nbad[n] = 0                      # the wrapped end, in the side batch the kernel hashes
    dk, do = dev(buf, offs)
    ndk, ndbo = dev(nbuf, nbad)
    with pkg.Filter(9585058377, 6) as f:
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        dig = torch.empty((n, 4), dtype=torch.int32, device="cuda")
        f.include_hash_dev(dk.data_ptr(), do.data_ptr(), n, out.data_ptr(), ndk.data_ptr(), ndbo.data_ptr(), n,
                           dig.data_ptr())
        expect_einval_once(pkg, f)
        words = dig.cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(words[n - 1], empty_words())


def test_lua_include_many_dev_bad_offsets_einval(pkg):
    n = 1000
    _, buf, offs = batch(n, seed=5)
    bad = offs.copy()
    bad[501] = bad[500] - 2
    dk, do = dev(buf, offs)
    _, dbo = dev(buf, bad)
    with pkg.LuaFilter(1000, 0.01) as f:
        f.insert_many_dev(dk.data_ptr(), do.data_ptr(), n)
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        f.include_many_dev(dk.data_ptr(), dbo.data_ptr(), n, out.data_ptr())
        torch.cuda.synchronize()
        with pytest.raises(pkg.ArgumentError, match="key offsets were inconsistent"):   # the next call
            f.include_many_dev(dk.data_ptr(), do.data_ptr(), n, out.data_ptr())
        f.include_many_dev(dk.data_ptr(), do.data_ptr(), n, out.data_ptr())
        torch.cuda.synchronize()
        assert out.cpu().numpy().all()
