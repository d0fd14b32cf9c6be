"""Key marshalling: Ruby ``data.to_s`` semantics and packing into (bytes, offsets).

The reference hashes ``data.to_s`` (lib/bloomfilter_driver/ruby.rb:42), so a
key's bytes depend on its Ruby class.  ``to_s`` below reproduces that for the
Python types that correspond to Ruby's:

=============  ==========================  ==================================
Python         Ruby analogue               bytes hashed
=============  ==========================  ==================================
bytes          String (binary)             as is
str            String (UTF-8)              UTF-8 encoding
int            Integer                     decimal, e.g. ``42`` -> ``b"42"``
bool           true / false                ``b"true"`` / ``b"false"``
None           nil                         ``b""``
float          Float                       Ruby ``Float#to_s`` (see below)
=============  ==========================  ==================================

Anything else raises TypeError (Ruby would call an arbitrary ``#to_s``).
"""
from __future__ import annotations

import math
from typing import Iterable, Tuple

import numpy as np


def ruby_float_to_s(x: float) -> str:
    """Ruby ``Float#to_s`` (flo_to_s): shortest round-trip digits, fixed notation
    for decimal exponents -4 < e <= 16, otherwise ``d.ddde+XX``."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))                      # shortest round-trip representation
    mant, _, exp = r.partition("e")
    digits = mant.replace(".", "")
    point = mant.index(".") if "." in mant else len(mant)
    decpt = point + (int(exp) if exp else 0)
    stripped = digits.lstrip("0")
    decpt -= len(digits) - len(stripped)
    digits = stripped.rstrip("0") or "0"
    if 0 < decpt <= 16:
        if len(digits) <= decpt:
            return sign + digits + "0" * (decpt - len(digits)) + ".0"
        return sign + digits[:decpt] + "." + digits[decpt:]
    if -4 < decpt <= 0:
        return sign + "0." + "0" * (-decpt) + digits
    e = decpt - 1
    frac = digits[1:] or "0"
    return "%s%s.%se%s%02d" % (sign, digits[0], frac, "+" if e >= 0 else "-", abs(e))


def to_s(data) -> bytes:
    """Bytes the reference would hash for ``data`` (``data.to_s``, ruby.rb:42)."""
    if isinstance(data, bytes):
        return data
    if isinstance(data, (bytearray, memoryview)):
        return bytes(data)
    if isinstance(data, str):
        return data.encode("utf-8")
    if data is None:
        return b""
    if isinstance(data, bool):
        return b"true" if data else b"false"
    if isinstance(data, (int, np.integer)):
        return str(int(data)).encode()
    if isinstance(data, (float, np.floating)):
        return ruby_float_to_s(float(data)).encode()
    raise TypeError("unsupported key type %s (expected bytes/str/int/float/bool/None)" % type(data).__name__)


def pack(keys: Iterable) -> Tuple[np.ndarray, np.ndarray]:
    """Pack keys into (uint8 key bytes, uint64 offsets[n+1])."""
    if isinstance(keys, np.ndarray) and keys.dtype.kind in "iu":
        return pack_decimal(keys)
    bs = [to_s(k) for k in keys]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        np.cumsum(np.fromiter((len(b) for b in bs), dtype=np.uint64, count=len(bs)), out=offs[1:])
    buf = np.frombuffer(b"".join(bs), dtype=np.uint8).copy() if bs else np.zeros(0, np.uint8)
    return buf, offs


def pack_decimal(values: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Vectorised ``Integer#to_s`` + pack for an integer array (the bench's key family D)."""
    v = np.asarray(values).reshape(-1)
    n = len(v)
    if n == 0:
        return np.zeros(0, np.uint8), np.zeros(1, np.uint64)
    neg = (v < 0) if v.dtype.kind == "i" else np.zeros(n, bool)
    if v.dtype.kind == "i":
        mag = np.abs(v.astype(np.int64)).astype(np.uint64)
        mag[v == np.iinfo(np.int64).min] = np.uint64(1) << np.uint64(63)
    else:
        mag = v.astype(np.uint64)
    pow10 = np.array([10 ** i for i in range(20)], dtype=np.uint64)
    ndig = np.searchsorted(pow10, mag, side="right").astype(np.int64)
    ndig[ndig == 0] = 1
    width = int(ndig.max()) + int(neg.any())
    # Right-aligned digit matrix, then a row-major boolean compaction.
    mat = np.empty((n, width), dtype=np.uint8)
    m = mag.copy()
    for j in range(width - 1, -1, -1):
        mat[:, j] = (m % np.uint64(10)).astype(np.uint8) + 48
        m //= np.uint64(10)
    lens = ndig + neg
    col = np.arange(width)
    keep = col[None, :] >= (width - lens)[:, None]
    if neg.any():
        mat[np.nonzero(neg)[0], width - lens[neg]] = ord("-")
    buf = mat[keep]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return buf, offs


def unpack(buf: np.ndarray, offs: np.ndarray, i: int) -> bytes:
    return bytes(buf[int(offs[i]):int(offs[i + 1])])
