"""In-memory stand-in for the Redis server commands the reference drivers use.

The reference specs run against a live redis-server (spec/redis_bloomfilter_spec.rb:26);
none is available here, so the tests and examples use this model of the
string commands with Redis's exact semantics:

* SETBIT/GETBIT: offset o -> byte o >> 3, bit 0x80 >> (o & 7); SETBIT grows the
  string zero-padded to o/8 + 1 bytes and returns the old bit; GETBIT past the
  end (or on a missing key) is 0; offsets must be < 2^32 (512 MB strings).
* SETRANGE grows zero-padded and keeps the TTL; SET replaces value and clears the TTL.
* EXPIRE/TTL with lazy expiry against an injectable clock.

Method names follow redis-py (``delete`` for DEL), so a real ``redis.Redis``
client can be passed wherever a ``FakeRedis`` is.
"""
from __future__ import annotations

import fnmatch
import math
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

PROTO_MAX_BULK = 512 * 1024 * 1024   # stock Redis string cap (offset < 2^32 bits)


class ResponseError(Exception):
    """Mirror of redis' error replies."""


class FakeRedis:
    def __init__(self, version: str = "7.2.0", clock: Callable[[], float] = time.monotonic,
                 max_string: int = PROTO_MAX_BULK):
        self._data: Dict[str, bytearray] = {}
        self._exp: Dict[str, float] = {}
        self._clock = clock
        self._version = version
        self._max = max_string
        self._lock = threading.RLock()
        self.calls: List[Tuple[str, str]] = []   # (command, key) log for tests
        self.bytes_in = 0                        # payload bytes received by SET/SETRANGE

    # -- internals
    def _key(self, name) -> str:
        return name.decode() if isinstance(name, bytes) else str(name)

    def _alive(self, k: str) -> bool:
        exp = self._exp.get(k)
        if exp is not None and self._clock() >= exp:
            self._data.pop(k, None)
            self._exp.pop(k, None)
        return k in self._data

    def _grow(self, k: str, size: int) -> bytearray:
        if size > self._max:
            raise ResponseError("ERR string exceeds maximum allowed size (proto-max-bulk-len)")
        buf = self._data.setdefault(k, bytearray())
        if len(buf) < size:
            buf.extend(b"\0" * (size - len(buf)))
        return buf

    # -- server
    def info(self, section=None) -> dict:
        return {"redis_version": self._version}

    def flushdb(self):
        with self._lock:
            self._data.clear()
            self._exp.clear()
        return True

    # -- bit commands
    def setbit(self, name, offset: int, value: int) -> int:
        k = self._key(name)
        offset = int(offset)
        if offset < 0 or offset >= self._max * 8:
            raise ResponseError("ERR bit offset is not an integer or out of range")
        with self._lock:
            self.calls.append(("SETBIT", k))
            self._alive(k)
            buf = self._grow(k, (offset >> 3) + 1)
            mask = 0x80 >> (offset & 7)
            old = 1 if buf[offset >> 3] & mask else 0
            if value:
                buf[offset >> 3] |= mask
            else:
                buf[offset >> 3] &= ~mask & 0xFF
            return old

    def getbit(self, name, offset: int) -> int:
        k = self._key(name)
        offset = int(offset)
        if offset < 0 or offset >= self._max * 8:
            raise ResponseError("ERR bit offset is not an integer or out of range")
        with self._lock:
            self.calls.append(("GETBIT", k))
            if not self._alive(k):
                return 0
            buf = self._data[k]
            if (offset >> 3) >= len(buf):
                return 0
            return 1 if buf[offset >> 3] & (0x80 >> (offset & 7)) else 0

    # -- string commands
    def get(self, name) -> Optional[bytes]:
        k = self._key(name)
        with self._lock:
            self.calls.append(("GET", k))
            return bytes(self._data[k]) if self._alive(k) else None

    def set(self, name, value) -> bool:
        k = self._key(name)
        v = value.encode() if isinstance(value, str) else bytes(value)
        if len(v) > self._max:
            raise ResponseError("ERR string exceeds maximum allowed size (proto-max-bulk-len)")
        with self._lock:
            self.calls.append(("SET", k))
            self.bytes_in += len(v)
            self._data[k] = bytearray(v)
            self._exp.pop(k, None)
            return True

    def setrange(self, name, offset: int, value) -> int:
        k = self._key(name)
        v = value.encode() if isinstance(value, str) else bytes(value)
        with self._lock:
            self.calls.append(("SETRANGE", k))
            self.bytes_in += len(v)
            alive = self._alive(k)
            if not v:
                return len(self._data[k]) if alive else 0
            buf = self._grow(k, int(offset) + len(v))
            buf[int(offset):int(offset) + len(v)] = v
            return len(buf)

    def getrange(self, name, start: int, end: int) -> bytes:
        k = self._key(name)
        with self._lock:
            self.calls.append(("GETRANGE", k))
            if not self._alive(k):
                return b""
            buf = self._data[k]
            n = len(buf)
            if start < 0:
                start = max(n + start, 0)
            if end < 0:
                end = n + end
            end = min(end, n - 1)
            if start > end or n == 0:
                return b""
            return bytes(buf[start:end + 1])

    def incr(self, name, amount: int = 1) -> int:
        """INCR / INCRBY: a missing key counts from 0; the TTL is kept."""
        k = self._key(name)
        with self._lock:
            self.calls.append(("INCR", k))
            cur = int(self._data[k].decode()) if self._alive(k) else 0
            cur += int(amount)
            self._data[k] = bytearray(str(cur).encode())
            return cur

    def strlen(self, name) -> int:
        k = self._key(name)
        with self._lock:
            return len(self._data[k]) if self._alive(k) else 0

    # -- keyspace
    def delete(self, *names) -> int:
        n = 0
        with self._lock:
            for name in names:
                k = self._key(name)
                self.calls.append(("DEL", k))
                if self._alive(k):
                    n += 1
                self._data.pop(k, None)
                self._exp.pop(k, None)
        return n

    def exists(self, *names) -> int:
        with self._lock:
            return sum(1 for nm in names if self._alive(self._key(nm)))

    def keys(self, pattern: str = "*") -> List[bytes]:
        with self._lock:
            return [k.encode() for k in list(self._data) if self._alive(k) and fnmatch.fnmatchcase(k, pattern)]

    def expire(self, name, seconds) -> bool:
        k = self._key(name)
        with self._lock:
            self.calls.append(("EXPIRE", k))
            if not self._alive(k):
                return False
            if seconds <= 0:
                self._data.pop(k, None)
                self._exp.pop(k, None)
                return True
            self._exp[k] = self._clock() + float(seconds)
            return True

    def ttl(self, name) -> int:
        k = self._key(name)
        with self._lock:
            if not self._alive(k):
                return -2
            exp = self._exp.get(k)
            if exp is None:
                return -1
            return int(math.ceil(exp - self._clock() - 1e-9))

    def pttl(self, name) -> int:
        k = self._key(name)
        with self._lock:
            if not self._alive(k):
                return -2
            exp = self._exp.get(k)
            if exp is None:
                return -1
            return int(math.ceil((exp - self._clock()) * 1000 - 1e-6))

    def persist(self, name) -> bool:
        k = self._key(name)
        with self._lock:
            return self._exp.pop(k, None) is not None if self._alive(k) else False


_current: Optional[FakeRedis] = None


def current() -> FakeRedis:
    """Process-wide default connection — the analogue of ``Redis.current``
    (lib/redis/bloomfilter.rb:18).  There is no redis-server here, so it is
    an in-memory FakeRedis."""
    global _current
    if _current is None:
        _current = FakeRedis()
    return _current
