"""CPU oracle for the redis-bloomfilter hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker (or the timed CPU
baseline).  The product package ``redis-bloomfilter_amd/`` never imports it and
has no CPU fallback.

Two independent restatements of the reference ruby driver live here:

* ``COracle`` — ctypes binding of ``oracle/bf_oracle.c`` (own SHA-1, OpenMP
  batch loops).  Fast enough for the parity tests at 10^5-10^7 keys and for
  the CPU baseline.
* ``py_*`` functions — pure Python over ``hashlib.sha1`` (an SHA-1 written by
  someone else), used to pin the C restatement and to generate the golden
  fixtures in ``tests/golden/``.

Reference lines restated (paths relative to the reference repository):
  lib/redis/bloomfilter.rb:50-52   optimal_m
  lib/redis/bloomfilter.rb:54-58   optimal_k
  lib/bloomfilter_driver/ruby.rb:41-55  indexes_for
  lib/bloomfilter_driver/ruby.rb:15-17,57-63  insert / set (EXPIRE iff !found && expire)
  lib/bloomfilter_driver/ruby.rb:20-30  include?
  lib/bloomfilter_driver/ruby.rb:33-35  clear (DEL)
  lib/bloomfilter_driver/ruby_test.rb:43-61  the RubyTest hash engines (py_engine_indexes)
"""
from __future__ import annotations

import ctypes
import hashlib
import math
import os
import subprocess
from typing import Iterable, List, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libbforacle.so")

# ----------------------------------------------------------------- sizing --


def ruby_round(x: float) -> int:
    """Ruby Float#round: half away from zero (Python's round() is half-even)."""
    if math.isnan(x) or math.isinf(x):
        raise FloatingPointError("FloatDomainError: %r" % x)
    r = math.floor(abs(x) + 0.5)
    return int(r) if x >= 0 else -int(r)


def py_optimal_m(n, p) -> int:
    """bloomfilter.rb:50-52 ``(-1 * n * Math.log(p) / (Math.log(2)**2)).round``."""
    return ruby_round((-1 * n) * math.log(p) / (math.log(2) ** 2))


def py_optimal_k(n, m) -> int:
    """bloomfilter.rb:54-58; Integer n -> floor division, Float n -> float division."""
    if isinstance(n, int) and isinstance(m, int):
        q = m // n
    else:
        q = m / n
    h = ruby_round(math.log(2) * q)
    if h == 0:
        h += 1
    return h


# ---------------------------------------------------------------- indexes --


def ruby_to_s(data) -> bytes:
    """``data.to_s`` for the key types the reference tests use (String, Integer)."""
    if isinstance(data, bytes):
        return data
    if isinstance(data, bool) or data is None:
        raise TypeError("oracle handles String/Integer keys only")
    if isinstance(data, int):
        return str(data).encode()
    if isinstance(data, str):
        return data.encode("utf-8")
    raise TypeError("oracle handles String/Integer keys only")


def py_digest_words(key: bytes) -> List[int]:
    """ruby.rb:42-47: hexdigest sliced into 4 big-endian 32-bit words."""
    sha = hashlib.sha1(key).hexdigest()
    return [int(sha[0:8], 16), int(sha[8:16], 16), int(sha[16:24], 16), int(sha[24:32], 16)]


def py_indexes(key, m: int, k: int) -> List[int]:
    """ruby.rb:41-55 ``indexes_for`` (pure Python, arbitrary precision like Ruby)."""
    h = py_digest_words(ruby_to_s(key))
    return [(h[i % 2] + i * h[2 + (((i + (i % 2)) % 4) // 2)]) % m for i in range(k)]


RFC1321_MD5 = {   # RFC 1321 appendix A.5 test suite
    "": "d41d8cd98f00b204e9800998ecf8427e",
    "a": "0cc175b9c0f1b6a831c399e269772661",
    "abc": "900150983cd24fb0d6963f7d28e17f72",
    "message digest": "f96b697d7cb7938d525a2f31aaf161d0",
    "abcdefghijklmnopqrstuvwxyz": "c3fcd3d76192e4007dfb496cca67e13b",
    "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789": "d174ab98d277d9f5a5611c2c9f419d9f",
    "1234567890" * 8: "57edf4a22be3c955ac49da2e2107b67a",
}


def py_engine_indexes(key, m: int, k: int, engine: str) -> List[int]:
    """ruby_test.rb:43-61: ``Digest::<E>.hexdigest("#{i}-#{data}").to_i(16) % bits`` for
    i in 0...k, ``data`` = ``key.to_s``; crc32 (``:52``) raises, as ``Integer#to_i(16)`` does."""
    if engine == "crc32":
        raise ArgumentError_("wrong number of arguments (given 1, expected 0)")
    f = {"md5": hashlib.md5, "sha1": hashlib.sha1}[engine]
    data = ruby_to_s(key)
    return [int(f(b"%d-" % i + data).hexdigest(), 16) % m for i in range(k)]


class ArgumentError_(Exception):
    """Ruby's ArgumentError, raised by the restated engine_crc32."""


def reach_bits(m: int, k: int) -> int:
    return min(m, k * 0xFFFFFFFF + 1)


# ------------------------------------------------------------ Redis model --


class PyBitstring:
    """A Redis string under SETBIT/GETBIT (MSB-first; grows to offset/8 + 1)."""

    def __init__(self, data: bytes = b""):
        self.buf = bytearray(data)

    def setbit(self, o: int, v: int) -> int:
        byte = o >> 3
        if byte >= len(self.buf):
            self.buf.extend(b"\0" * (byte + 1 - len(self.buf)))
        mask = 0x80 >> (o & 7)
        old = 1 if self.buf[byte] & mask else 0
        if v:
            self.buf[byte] |= mask
        else:
            self.buf[byte] &= ~mask & 0xFF
        return old

    def getbit(self, o: int) -> int:
        byte = o >> 3
        if byte >= len(self.buf):
            return 0
        return 1 if self.buf[byte] & (0x80 >> (o & 7)) else 0

    def value(self) -> bytes:
        return bytes(self.buf)


class RubyDriverRestatement:
    """lib/bloomfilter_driver/ruby.rb restated over a redis-like client.

    The client needs ``setbit``, ``getbit``, ``expire`` and ``delete``.  Used
    by the interop tests: a filter written here must read identically through
    the HIP driver and vice versa.
    """

    def __init__(self, options: dict):
        self.options = options
        self.redis = options.get("redis")

    def insert(self, data, expire=None):  # ruby.rb:15-17
        self._set(data, expire)

    def include(self, key) -> bool:  # ruby.rb:20-30
        idx = py_indexes(key, self.options["bits"], self.options["hashes"])
        name = self.options["key_name"]
        if self.redis.getbit(name, idx[0]) == 0:
            return False
        return all(self.redis.getbit(name, i) == 1 for i in idx[1:])

    def clear(self):  # ruby.rb:33-35
        self.redis.delete(self.options["key_name"])

    def _set(self, key, expire):  # ruby.rb:57-63
        name = self.options["key_name"]
        changed = [self.redis.setbit(name, i, 1)
                   for i in py_indexes(key, self.options["bits"], self.options["hashes"])]
        found = 0 not in changed
        if not found and expire is not None and expire is not False:   # Ruby truthiness: 0 expires
            self.redis.expire(name, expire)


# ------------------------------------------------------- C oracle (ctypes) --

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build() -> str:
    """Compile oracle/bf_oracle.c (gcc) if needed; returns the .so path."""
    src = os.path.join(HERE, "bf_oracle.c")
    if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def pack_keys(keys: Iterable) -> tuple:
    """Pack keys into (uint8 bytes, uint64 offsets[n+1])."""
    bs = [ruby_to_s(k) for k in keys]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        offs[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bs), dtype=np.uint8) if bs else np.zeros(0, np.uint8)
    return np.ascontiguousarray(buf), offs


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


class COracle:
    def __init__(self, path: str | None = None):
        self.lib = ctypes.CDLL(path or build())
        L = self.lib
        L.bfo_sha1.argtypes = [_u8p, ctypes.c_uint64, _u8p]
        L.bfo_optimal_m.argtypes = [ctypes.c_double, ctypes.c_double]
        L.bfo_optimal_m.restype = ctypes.c_int64
        L.bfo_optimal_k_int.argtypes = [ctypes.c_int64, ctypes.c_int64]
        L.bfo_optimal_k_int.restype = ctypes.c_int64
        L.bfo_optimal_k_float.argtypes = [ctypes.c_double, ctypes.c_int64]
        L.bfo_optimal_k_float.restype = ctypes.c_int64
        L.bfo_indexes.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, _u64p]
        L.bfo_indexes_many.argtypes = [_u8p, _u64p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, _u64p]
        L.bfo_reach_bits.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
        L.bfo_reach_bits.restype = ctypes.c_uint64
        L.bfo_insert_many.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, _u8p, _u64p,
                                      ctypes.c_uint64, _u8p, _u8p]
        L.bfo_include_many.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, _u8p, _u64p,
                                       ctypes.c_uint64, _u8p]
        L.bfo_insert_many_omp.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, _u8p, _u64p,
                                          ctypes.c_uint64, ctypes.c_int]
        L.bfo_include_many_omp.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, _u8p, _u64p,
                                           ctypes.c_uint64, _u8p, ctypes.c_int]
        L.bfo_redis_len.argtypes = [_u8p, ctypes.c_uint64]
        L.bfo_redis_len.restype = ctypes.c_uint64
        L.bfo_max_threads.restype = ctypes.c_int

    # -- scalar helpers
    def sha1(self, msg: bytes) -> bytes:
        a = np.frombuffer(msg, dtype=np.uint8) if msg else np.zeros(1, np.uint8)
        out = np.zeros(20, np.uint8)
        self.lib.bfo_sha1(_p(a, _u8p), len(msg), _p(out, _u8p))
        return out.tobytes()

    def optimal_m(self, n, p) -> int:
        return int(self.lib.bfo_optimal_m(float(n), float(p)))

    def optimal_k(self, n, m) -> int:
        if isinstance(n, int):
            return int(self.lib.bfo_optimal_k_int(n, m))
        return int(self.lib.bfo_optimal_k_float(float(n), m))

    def indexes(self, key, m: int, k: int) -> List[int]:
        b = ruby_to_s(key)
        a = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8)
        out = np.zeros(k, np.uint64)
        self.lib.bfo_indexes(_p(a, _u8p), len(b), m, k, _p(out, _u64p))
        return [int(x) for x in out]

    def indexes_many(self, keys: np.ndarray, offs: np.ndarray, m: int, k: int) -> np.ndarray:
        n = len(offs) - 1
        out = np.zeros(max(n * k, 1), np.uint64)
        kb = keys if len(keys) else np.zeros(1, np.uint8)
        self.lib.bfo_indexes_many(_p(kb, _u8p), _p(offs, _u64p), n, m, k, _p(out, _u64p))
        return out[: n * k].reshape(n, k)

    def reach_bits(self, m: int, k: int) -> int:
        return int(self.lib.bfo_reach_bits(m, k))

    # -- batch, on a host bitset of ceil(reach/8) bytes (Redis byte order)
    def new_bitset(self, m: int, k: int) -> np.ndarray:
        return np.zeros((self.reach_bits(m, k) + 7) // 8, dtype=np.uint8)

    def insert_many(self, bits: np.ndarray, m: int, k: int, keys: np.ndarray, offs: np.ndarray,
                    per_key: bool = False):
        n = len(offs) - 1
        pk = np.zeros(max(n, 1), np.uint8)
        anyn = np.zeros(1, np.uint8)
        kb = keys if len(keys) else np.zeros(1, np.uint8)
        self.lib.bfo_insert_many(_p(bits, _u8p), m, k, _p(kb, _u8p), _p(offs, _u64p), n,
                                 _p(pk, _u8p), _p(anyn, _u8p))
        return bool(anyn[0]), pk[:n]

    def include_many(self, bits: np.ndarray, m: int, k: int, keys: np.ndarray,
                     offs: np.ndarray) -> np.ndarray:
        n = len(offs) - 1
        out = np.zeros(max(n, 1), np.uint8)
        kb = keys if len(keys) else np.zeros(1, np.uint8)
        self.lib.bfo_include_many(_p(bits, _u8p), m, k, _p(kb, _u8p), _p(offs, _u64p), n,
                                  _p(out, _u8p))
        return out[:n]

    def insert_many_omp(self, bits, m, k, keys, offs, threads: int):
        self.lib.bfo_insert_many_omp(_p(bits, _u8p), m, k, _p(keys, _u8p), _p(offs, _u64p),
                                     len(offs) - 1, threads)

    def include_many_omp(self, bits, m, k, keys, offs, threads: int) -> np.ndarray:
        out = np.zeros(max(len(offs) - 1, 1), np.uint8)
        self.lib.bfo_include_many_omp(_p(bits, _u8p), m, k, _p(keys, _u8p), _p(offs, _u64p),
                                      len(offs) - 1, _p(out, _u8p), threads)
        return out[: len(offs) - 1]

    def redis_string(self, bits: np.ndarray) -> bytes:
        n = int(self.lib.bfo_redis_len(_p(bits, _u8p), len(bits)))
        return bits[:n].tobytes()

    def max_threads(self) -> int:
        return int(self.lib.bfo_max_threads())


def sha1_hex(b: bytes) -> str:
    return hashlib.sha1(b).hexdigest()


__all__ = [
    "COracle", "PyBitstring", "RubyDriverRestatement", "build", "pack_keys", "py_indexes",
    "py_optimal_m", "py_optimal_k", "py_digest_words", "reach_bits", "ruby_round", "ruby_to_s",
    "sha1_hex",
]
