"""The region-set buffer format (include/bfhip.h, bf_binned.hip) on the host: the test
reader (tests/sets_codec.py) inverts a host-side encoding of the same layout, in Elias-Fano
and bitmap form, and the capacity bound holds for the densest and most even batches (the
even split is the worst case of the concave per-region size)."""
import numpy as np
import pytest

import sets_codec


@pytest.mark.parametrize("rl", [18, 19])
def test_round_trip(rl):
    rng = np.random.default_rng(rl)
    U = 1 << rl
    sets = {}
    for r, n in enumerate([0, 1, 2, 7, 100, 2048, 5000, U // 8, U // 4, U // 2, U - 3, U]):
        if n:
            sets[r] = np.sort(rng.choice(U, size=n, replace=False)).astype(np.uint64)
    words = sets_codec.encode(sets, rl, 12)
    got = sets_codec.decode(words)
    assert sorted(got) == sorted(sets)
    for r in sets:
        np.testing.assert_array_equal(got[r], sets[r])


@pytest.mark.parametrize("n_keys,k,bitset", [
    (1 << 24, 13, 6_977_001_472),     # 10B@0.01 %: the replicated step's batch
    (1 << 24, 6, 1_198_132_480),      # the north-star filter
    (40_000, 6, 1_198_336),           # 1M@1 %: dense (bitmap regions)
    (100, 10, 179_719_936),           # sparse
])
def test_capacity_bounds_even_batches(n_keys, k, bitset):
    """An even spread of n k distinct offsets over the regions (the bound's worst case) fits
    the capacity; measured here on a few regions' actual set sizes, scaled to all."""
    rl = 19
    U = 1 << rl
    R = -(-(bitset * 8) // U)
    per = n_keys * k / R
    n = max(1, min(U, int(round(per))))
    rng = np.random.default_rng(1)
    xs = np.sort(rng.choice(U, size=n, replace=False)).astype(np.uint64)
    one = len(sets_codec.encode({0: xs}, rl, 1)) - (4 + 2 + 63) // 64 * 64
    need = (4 + 2 * R + 63) // 64 * 64 + one * min(R, n_keys * k)
    assert need <= sets_codec.capacity_words(bitset, rl, n_keys, k)
