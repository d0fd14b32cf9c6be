"""The Lua driver's scalable layout on the GPU against the restated
scripts (oracle/lua_oracle.py: vendor/assets/lua/add.lua, check.lua) run over
FakeRedis: the count, every layer's Redis string, each key's INCR flag and every
include? answer must match exactly.
"""
import lua_oracle as L
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def script_run(pkg, keys, entries, precision, key="lbf", r=None):
    r = r or pkg.FakeRedis()
    flags = [L.add(r, key, entries, precision, k) for k in keys]
    return r, np.array(flags, dtype=bool)


def layers_of(r, key):
    out = {}
    n = 1
    while r.exists("%s:%d" % (key, n)):
        out[n] = r.get("%s:%d" % (key, n))
        n += 1
    return out


@pytest.mark.parametrize("entries,precision,nkeys,span,batches", [
    (100, 0.01, 900, 700, 1),          # 4 layers, many repeats, one batch
    (100, 0.01, 900, 700, 7),          # the same keys in uneven batches
    (1000, 0.02, 5000, 10**9, 3),      # distinct keys, 3 layers
    (50, 0.2, 2000, 3000, 2),          # tiny filter, low k, dense layers
    (10_000, 0.001, 100_000, 10**12, 1),   # 4 layers of a bigger filter
])
def test_lua_insert_include_match_scripts(pkg, entries, precision, nkeys, span, batches):
    rng = np.random.default_rng(11)
    keys = [int(v) for v in rng.integers(0, span, nkeys)]
    r, want_flags = script_run(pkg, keys, entries, precision)
    cuts = np.linspace(0, nkeys, batches + 1).astype(int)
    cuts[1:-1] += rng.integers(-7, 8, batches - 1) if batches > 1 else 0
    got_flags = []
    with pkg.LuaFilter(entries, precision) as f:
        for a, b in zip(cuts[:-1], cuts[1:]):
            buf, offs = pkg.keys.pack(keys[a:b])
            pk, touched = f.insert_many(buf, offs)
            got_flags.append(pk.astype(bool))
        np.testing.assert_array_equal(np.concatenate(got_flags), want_flags)
        assert f.count == int(r.get("lbf:count"))
        want_layers = layers_of(r, "lbf")
        assert f.layers == len(want_layers) and len(want_layers) >= 2
        for n, s in want_layers.items():
            assert f.export_layer(n) == s, n
        probe = keys[: nkeys // 2] + ["fresh-%d" % i for i in range(nkeys // 2)]
        pb, po = pkg.keys.pack(probe)
        got = f.include_many(pb, po).astype(bool)
        want = np.array([L.check(r, "lbf", entries, precision, k) for k in probe])
        np.testing.assert_array_equal(got, want)
        assert got[: nkeys // 2].all()


@pytest.mark.parametrize("entries,precision,nkeys,span,batches", [
    (100, 0.01, 900, 700, 3),          # repeats, layer cuts inside a batch
    (1000, 0.02, 5000, 10**9, 1),      # distinct keys, 3 layers in one call
    (10_000, 0.001, 100_000, 10**12, 2),
])
def test_lua_device_entry_points_match_scripts(pkg, entries, precision, nkeys, span, batches):
    """bf_lua_insert_many_dev / bf_lua_include_many_dev (device keys, the caller's stream, flags
    and answers left on the device, the INCRs summed on the device) against the scripts: the
    same per-key INCR flags, count, layer strings and include? answers; per-layer kernel times
    from bf_lua_profile."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(13)
    keys = [int(v) for v in rng.integers(0, span, nkeys)]
    r, want_flags = script_run(pkg, keys, entries, precision)
    cuts = np.linspace(0, nkeys, batches + 1).astype(int)
    st = torch.cuda.current_stream().cuda_stream
    got_flags = []
    with pkg.LuaFilter(entries, precision) as f:
        f.profile(True)
        for a, b in zip(cuts[:-1], cuts[1:]):
            buf, offs = pkg.keys.pack(keys[a:b])
            kb = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).cuda()
            ko = torch.from_numpy(offs.view(np.int64)).cuda()
            flags = torch.zeros(b - a, dtype=torch.uint8, device="cuda")
            f.insert_many_dev(kb.data_ptr(), ko.data_ptr(), b - a, flags.data_ptr(), stream=st)
            got_flags.append(flags.cpu().numpy().astype(bool))
        np.testing.assert_array_equal(np.concatenate(got_flags), want_flags)
        assert f.count == int(r.get("lbf:count"))
        want_layers = layers_of(r, "lbf")
        assert f.layers == len(want_layers) and len(want_layers) >= 2
        for n, s in want_layers.items():
            assert f.export_layer(n) == s, n
        probe = keys[: nkeys // 2] + ["fresh-%d" % i for i in range(nkeys // 2)]
        pb, po = pkg.keys.pack(probe)
        # an odd device address: the kernels realign the key bytes
        kb = torch.zeros(len(pb) + 19, dtype=torch.uint8, device="cuda")
        kb[3: 3 + len(pb)] = torch.from_numpy(pb).cuda()
        ko = torch.from_numpy(po.view(np.int64)).cuda()
        out = torch.empty(len(probe), dtype=torch.uint8, device="cuda")
        f.include_many_dev(kb.data_ptr() + 3, ko.data_ptr(), len(probe), out.data_ptr(), stream=st)
        got = out.cpu().numpy().astype(bool)
        want = np.array([L.check(r, "lbf", entries, precision, k) for k in probe])
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(got, f.include_many(pb, po).astype(bool))   # = the host path
        prof = f.profile_read()
        assert "lua_check" in prof and "lua_seq_candidates[L1]" in prof and "lua_seq_mark[L2]" in prof


def test_hip_lua_driver_write_through_and_interop(pkg):
    """The driver's Redis keys equal the scripts' after the same inserts (lua.rb layout), a
    driver attached to the scripts' Redis answers like check.lua, and clear drops name:*."""
    rng = np.random.default_rng(12)
    keys = ["w%d" % v for v in rng.integers(0, 400, 500)]
    mine = pkg.FakeRedis()
    bf = pkg.Bloomfilter(size=100, error_rate=0.01, key_name="lbf", driver="hip-lua", redis=mine)
    bf.insert_many(keys[:300])
    bf.insert_many(keys[300:], 120)
    r, _ = script_run(pkg, keys, 100, 0.01)
    assert sorted(mine.keys("lbf:*")) == sorted(r.keys("lbf:*"))
    for k in r.keys("lbf:*"):
        assert mine.get(k) == r.get(k), k
    top = "lbf:%d" % len(layers_of(r, "lbf"))
    assert mine.ttl(top) > 0                      # add.lua:51-53 EXPIREs the layer written to
    other = pkg.Bloomfilter(size=100, error_rate=0.01, key_name="lbf", driver="hip-lua", redis=r)
    probe = keys[:100] + ["nope%d" % i for i in range(200)]
    np.testing.assert_array_equal(other.include_many(probe),
                                  [L.check(r, "lbf", 100, 0.01, k) for k in probe])
    bf.clear()
    assert mine.keys("lbf:*") == [] and not bf.include("w1")


def test_spec_scalable_filter_via_hip_lua(pkg):
    """spec/redis_bloomfilter_spec.rb:122-128 with driver 'hip-lua'."""
    bf = pkg.Bloomfilter(size=100, error_rate=0.02, key_name="__test_bf", driver="hip-lua", redis=pkg.FakeRedis())
    bf.clear()
    rng = np.random.default_rng(13)
    visited, errors = set(), 0
    for _ in range(150):
        a = int(rng.integers(0, 150))
        errors += bf.include(a) != (a in visited)
        visited.add(a)
        bf.insert(a)
    assert errors / 150 <= bf.options["error_rate"]
    bf.clear()


def test_hip_lua_per_key_setbit_replay(pkg):
    """Per-key inserts (the SETBIT-replay write-through, bf_lua_insert_many_changes): after
    every insert the driver's Redis keys equal what add.lua leaves, across layer growth, and
    the flipped bits reported are exactly the layers' new bits."""
    rng = np.random.default_rng(21)
    keys = ["p%d" % v for v in rng.integers(0, 300, 260)]
    mine, ref = pkg.FakeRedis(), pkg.FakeRedis()
    bf = pkg.Bloomfilter(size=50, error_rate=0.01, key_name="pk", driver="hip-lua", redis=mine)
    for i, key in enumerate(keys):
        got = bf.insert(key)
        want = L.add(ref, "pk", 50, 0.01, key)
        assert bool(got[0]) == bool(want), i
        assert sorted(mine.keys("pk:*")) == sorted(ref.keys("pk:*")), i
        for k in ref.keys("pk:*"):
            assert mine.get(k) == ref.get(k), (i, k)
    assert len(layers_of(ref, "pk")) >= 3   # the batch crossed layer thresholds
    f = bf.driver.filter
    before = {n: f.export_layer(n) for n in range(1, f.layers + 1)}
    b, o = pkg.keys.pack(["fresh%d" % i for i in range(40)])
    _, touched, flips = f.insert_many_changes(b, o)
    for n in range(1, f.layers + 1):
        old, new = before.get(n, b""), f.export_layer(n)
        old_bits = np.unpackbits(np.frombuffer(old.ljust(len(new), b"\0"), np.uint8)) if new else np.zeros(0, np.uint8)
        new_bits = np.unpackbits(np.frombuffer(new, np.uint8)) if new else np.zeros(0, np.uint8)
        want = set(np.flatnonzero(new_bits & ~old_bits).tolist())
        assert {o for (lay, o) in flips if lay == n} == want, n
    bf.driver.close()


def test_lua_changes_binned_batch_across_layers(pkg):
    """bf_lua_insert_many_changes on 6000 keys (the binned sequential form: 4096+ keys, layers
    of <= 2^27 bits) that fill layer 1 and run into layer 2 within one call: the flips reported
    are exactly the layers' new bits, one per bit, and the flags and layers match the script."""
    rng = np.random.default_rng(23)
    keys = ["b%d" % v for v in rng.integers(0, 9000, 6000)]
    r, want_flags = script_run(pkg, keys, 2000, 0.01)
    with pkg.LuaFilter(2000, 0.01) as f:
        b, o = pkg.keys.pack(keys)
        pk, touched, flips = f.insert_many_changes(b, o)
        np.testing.assert_array_equal(pk.astype(bool), want_flags)
        assert f.count == int(r.get("lbf:count")) and f.layers >= 2
        got = {}
        for lay, off in flips:
            got.setdefault(lay, []).append(off)
        for n, s in layers_of(r, "lbf").items():
            assert f.export_layer(n) == s, n
            offs = sorted(got.get(n, []))
            assert len(offs) == len(set(offs)), n    # each bit reported once
            bits = np.unpackbits(np.frombuffer(s, np.uint8))
            assert offs == np.flatnonzero(bits).tolist(), n
