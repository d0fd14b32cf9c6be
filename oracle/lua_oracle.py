"""TEST INFRASTRUCTURE — CPU restatement of the reference's Lua scripts.

vendor/assets/lua/add.lua and check.lua (run by lib/bloomfilter_driver/lua.rb
through EVALSHA), restated line by line over a redis-like client (GET, INCR,
SETBIT, GETBIT, EXPIRE).  Lua 5.1 numbers are IEEE doubles, so Python floats
reproduce the sizing math exactly; ``redis.sha1hex`` is FIPS SHA-1 (hashlib).
Only tests/ import this module (the checker of the ``hip-lua`` driver).

Parity: the layer sizes are pinned by SURVEY §8 f1 (1000 @ 0.01 -> 11027/7,
24940/8, 55652/9); no fixture of the reference pins the bitstrings, which are
pinned by this restatement alone ("parity unpinned" beyond the sizing).
"""
from __future__ import annotations

import hashlib
import math

LN2 = 0.69314718055995        # add.lua:14, the constant as written
LN2_SQ = 0.4804530139182      # add.lua:21


def layer_index(entries: float, count: float) -> int:
    """add.lua:13-15 / check.lua:9-11."""
    factor = math.ceil((entries + count) / entries)
    return math.ceil(math.log(factor) / LN2)


def layer_params(entries: float, precision: float, n: int):
    """add.lua:16-25 (check.lua:41-47): (bits, k) of layer n."""
    scale = math.pow(2, n - 1) * entries
    bits = math.floor(-(scale * math.log(precision * math.pow(0.5, n))) / LN2_SQ)
    k = math.floor(LN2 * bits / scale)
    return bits, k


def _h(data: bytes):
    """add.lua:3, 30-34: the four 32-bit words of sha1hex(data)."""
    hx = hashlib.sha1(data).hexdigest()
    return [int(hx[0:8], 16), int(hx[8:16], 16), int(hx[16:24], 16), int(hx[24:32], 16)]


def _probe(h, i: int) -> int:
    """add.lua:38 / check.lua:35: h[i % 2] + i * h[2 + ((i + i % 2) % 4) / 2] (i >= 1)."""
    return h[i % 2] + i * h[2 + ((i + i % 2) % 4) // 2]


def _b(data) -> bytes:
    return data if isinstance(data, bytes) else str(data).encode()


def add(redis, key: str, entries, precision, data, expire=None) -> bool:
    """add.lua:1-54; returns True iff the item was new (the INCR happened)."""
    entries, precision = float(entries), float(precision)
    h = _h(_b(data))
    countkey = key + ":count"
    raw = redis.get(countkey)
    count = 1 if raw is None else int(raw) + 1                         # :6-11
    index = layer_index(entries, count)                                # :13-15
    bits, k = layer_params(entries, precision, index)                  # :16-25
    lkey = "%s:%d" % (key, index)                                      # :17
    found = True
    for i in range(1, k + 1):                                          # :37-41
        if redis.setbit(lkey, _probe(h, i) % bits, 1) == 0:
            found = False
    if not found:                                                      # :48-54
        redis.incr(countkey)
        if expire is not None and expire is not False:   # tonumber(ARGV[4]) (add.lua:4): 0 is truthy in Lua
            redis.expire(lkey, expire)
    return not found


def check(redis, key: str, entries, precision, data) -> bool:
    """check.lua:1-61."""
    entries, precision = float(entries), float(precision)
    raw = redis.get(key + ":count")
    if raw is None:                                                    # :3-7
        return False
    count = int(raw)
    index = layer_index(entries, count)                                # :9-11
    h = _h(_b(data))
    _, maxk = layer_params(entries, precision, index)                  # :28-31
    b = [None] + [_probe(h, i) for i in range(1, maxk + 1)]            # :32-36
    for n in range(1, index + 1):                                      # :38-59
        bits, k = layer_params(entries, precision, n)
        if all(redis.getbit("%s:%d" % (key, n), b[i] % bits) for i in range(1, k + 1)):
            return True
    return False
