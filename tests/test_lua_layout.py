"""The Lua driver's scalable layout — CPU part: the restatement of
vendor/assets/lua/add.lua + check.lua (oracle/lua_oracle.py) pinned by the
SURVEY's layer sizes, and the C ABI's host-only sizing helpers against it.
"""
import lua_oracle as L
import numpy as np
import pytest


def test_layer_sizes_pinned():
    """1000 @ 0.01 -> layer 1: 11,027 bits / 7 hashes; 2: 24,940 / 8; 3: 55,652 / 9."""
    assert [L.layer_params(1000, 0.01, n) for n in (1, 2, 3)] == [(11027, 7), (24940, 8), (55652, 9)]


def test_layer_index_thresholds():
    """add.lua:13-15: layer n takes the counts up to (2^n - 1) * entries."""
    got = [L.layer_index(100.0, c) for c in (1, 100, 101, 300, 301, 700, 701, 1500, 1501)]
    assert got == [1, 1, 2, 2, 3, 3, 4, 4, 5]


@pytest.mark.parametrize("entries,precision", [(1000, 0.01), (100, 0.02), (10_000, 0.001), (1e6, 0.01),
                                               (1000.0, 0.05), (7, 0.3), (123456789, 1e-4)])
def test_abi_sizing_matches_scripts(pkg, entries, precision):
    lib = pkg._lib
    for n in range(1, 30):
        assert lib.lua_layer_params(entries, precision, n) == L.layer_params(float(entries), precision, n)
    rng = np.random.default_rng(3)
    counts = [1, 2, int(entries), int(entries) + 1] + [int(x) for x in rng.integers(1, 10 ** 12, 200)]
    counts += [(2 ** n - 1) * int(entries) + d for n in range(1, 20) for d in (0, 1)]
    for c in counts:
        assert lib.lua_index(entries, c) == L.layer_index(float(entries), c), c


def test_scripts_are_a_scalable_filter(pkg):
    """spec/redis_bloomfilter_spec.rb:122-128 on the restated scripts: 150 items into a
    100-item, 2 % filter, include? before every insert, error rate <= 2 %."""
    r = pkg.FakeRedis()
    rng = np.random.default_rng(5)
    visited, errors = set(), 0
    for _ in range(150):
        a = int(rng.integers(0, 150))
        errors += L.check(r, "__test_bf", 100, 0.02, a) != (a in visited)
        visited.add(a)
        L.add(r, "__test_bf", 100, 0.02, a)
    assert errors / 150 <= 0.02
    for i in range(300):   # past 100 new items the filter grows a second layer
        L.add(r, "__test_bf", 100, 0.02, "grow-%d" % i)
    assert int(r.get("__test_bf:count")) > 100 and r.exists("__test_bf:2") and not r.exists("__test_bf:4")


def test_hip_lua_driver_registered(pkg):
    assert pkg.driver_name("hip-lua") == "HipLua" and "HipLua" in pkg.DRIVERS
