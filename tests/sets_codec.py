"""Host-side reader of the region-set buffers bf_encode_region_sets_dev writes (include/bfhip.h)
— TEST INFRASTRUCTURE: it decodes a buffer independently of the device decoder, so the
tests can check the encoding itself against the oracle's offsets (ruby.rb:41-55).

Layout (uint32 words): [0] "BFRS", [1] region_log2, [2] regions R, [3] words used, [4 + r]
region r's first word (0: empty), [4 + R + r] its set's header word; a set is n | (l << 24), then ceil(n l / 32) words of low
bits (offset i's l bits at bit i l, LSB first) and ceil((n + (U >> l)) / 32) words of the upper
bitmap (offset i sets bit (x_i >> l) + i); l = 31: the region's bitmap in the bitset's own
word layout (offset x at bit (x & 31) ^ 7 of word x >> 5)."""
import numpy as np

MAGIC = 0x53524642


def header(words: np.ndarray):
    return int(words[0]), int(words[1]), int(words[2]), int(words[3])


def decode(buf) -> dict:
    """{region: sorted uint64 array of region-local offsets} of one set buffer."""
    w = np.frombuffer(bytes(buf), dtype=np.uint32) if not isinstance(buf, np.ndarray) else buf.view(np.uint32)
    magic, rl, R, used = header(w)
    assert magic == MAGIC, "not a region-set buffer"
    assert used <= len(w), "set buffer overflowed its capacity"
    U = 1 << rl
    out = {}
    for r in range(R):
        st = int(w[4 + r])
        if st == 0:
            assert int(w[4 + R + r]) == 0, "empty region with a header"
            continue
        hdr = int(w[st])
        assert int(w[4 + R + r]) == hdr, "header table disagrees with the set"
        n, l = hdr & 0xFFFFFF, hdr >> 24
        if l == 31:
            bm = w[st + 1: st + 1 + U // 32]
            bits = np.unpackbits(bm.view(np.uint8), bitorder="big")   # byte-major, MSB first = Redis order
            xs = np.flatnonzero(bits).astype(np.uint64)
            assert len(xs) == n, "bitmap set: count mismatch"
            out[r] = xs
            continue
        lw = (n * l + 31) // 32
        uw = (n + (U >> l) + 31) // 32
        lows_w = w[st + 1: st + 1 + lw]
        up_w = w[st + 1 + lw: st + 1 + lw + uw]
        up = np.unpackbits(up_w.view(np.uint8), bitorder="little")
        pos = np.flatnonzero(up)
        assert len(pos) == n, "upper bitmap: %d ones for %d offsets" % (len(pos), n)
        high = pos - np.arange(n)
        if l:
            lb = np.unpackbits(lows_w.view(np.uint8), bitorder="little")[: n * l].reshape(n, l)
            lows = (lb.astype(np.uint64) << np.arange(l, dtype=np.uint64)).sum(axis=1)
        else:
            lows = np.zeros(n, np.uint64)
        xs = (high.astype(np.uint64) << np.uint64(l)) | lows
        assert np.all(np.diff(xs.astype(np.int64)) > 0), "offsets not strictly ascending"
        out[r] = xs
    return out


def expected(idx: np.ndarray, region_log2: int) -> dict:
    """{region: sorted distinct region-local offsets} of a batch's probe offsets."""
    u = np.unique(np.asarray(idx, dtype=np.uint64).reshape(-1))
    reg = (u >> np.uint64(region_log2)).astype(np.int64)
    loc = u & np.uint64((1 << region_log2) - 1)
    out = {}
    if len(u):
        cut = np.flatnonzero(np.diff(reg)) + 1
        for part_r, part_x in zip(np.split(reg, cut), np.split(loc, cut)):
            out[int(part_r[0])] = part_x
    return out


def encode(sets: dict, region_log2: int, nregions: int) -> np.ndarray:
    """A set buffer holding `sets` ({region: sorted distinct offsets}), laid out as the device
    encode lays it out (regions in index order; the device's order is arbitrary)."""
    U = 1 << region_log2
    first = (4 + 2 * nregions + 63) // 64 * 64
    words = [0] * first
    words[0], words[1], words[2] = MAGIC, region_log2, nregions
    for r in range(nregions):
        xs = np.asarray(sets.get(r, []), dtype=np.uint64)
        n = len(xs)
        if n == 0:
            continue
        words[4 + r] = len(words)
        l = int(np.floor(np.log2(U // n))) if n else 0
        if n * l + n + (U >> l) > U:   # bitmap
            bits = np.zeros(U, np.uint8)
            bits[xs.astype(np.int64)] = 1
            words[4 + nregions + r] = n | (31 << 24)
            words.append(n | (31 << 24))
            words.extend(np.packbits(bits, bitorder="big").view(np.uint32).tolist())
            continue
        lw = (n * l + 31) // 32
        uw = (n + (U >> l) + 31) // 32
        lowbits = np.zeros(lw * 32, np.uint8)
        if l:
            lo = xs & np.uint64((1 << l) - 1)
            lowbits[: n * l] = ((lo[:, None] >> np.arange(l, dtype=np.uint64)) & np.uint64(1)).astype(np.uint8).reshape(-1)
        up = np.zeros(uw * 32, np.uint8)
        up[(xs >> np.uint64(l)).astype(np.int64) + np.arange(n)] = 1
        words[4 + nregions + r] = n | (l << 24)
        words.append(n | (l << 24))
        words.extend(np.packbits(lowbits, bitorder="little").view(np.uint32).tolist())
        words.extend(np.packbits(up, bitorder="little").view(np.uint32).tolist())
    words[3] = len(words)
    return np.asarray(words, dtype=np.uint32)


def capacity_words(bitset_bytes: int, region_log2: int, n_keys: int, k: int) -> int:
    """bf_sets_capacity_bytes / 4 (bf_binned.hip), restated for the host tests."""
    R = -(-(bitset_bytes * 8) // (1 << region_log2))
    U = float(1 << region_log2)
    N = min(float(n_keys * k), U * R)
    bits = 0.0
    if N > 0:
        bits = min(N * (np.log2(U * R / N) + 3.01), U * R) * 1.01 + 4096.0
    words = (4 + 2 * R + 63) // 64 * 64 + 4 * R + int(bits / 32.0) + 64
    return (words + 63) // 64 * 64
