"""``Redis::BloomfilterDriver::Hip`` — the MI355X driver, Python host mirror.

Plugs in exactly where lib/bloomfilter_driver/ruby.rb does (duck-typed
driver: ``__init__(options)``, ``redis`` attribute, ``insert``, ``include``,
``clear``) and adds ``insert_many`` / ``include_many``.  The filter lives in
HBM (one ``bf_handle``); Redis keeps the same bitstring the ruby driver writes:

* attach (``driver.redis = r``, bloomfilter.rb:45): if ``key_name`` exists it is
  imported (a filter written by the ruby driver is readable here) and its TTL
  is mirrored;
* ``sync='write_through'`` (default): an insert that flips a bit writes the
  64 KiB blocks of the string it changed back with SETRANGE (keeps the key's
  TTL, grows it like SETBIT would), then EXPIREs when ``expire`` is given —
  ruby.rb:61-62.  The device keeps a dirty-block map (``bf_track_dirty``), so a
  small batch into a multi-GB filter writes kilobytes, not the whole string;
* ``sync='manual'``: Redis is only touched by ``clear`` (DEL) and by explicit
  ``flush()`` / ``reload()``; ``flush()`` writes what changed since the last
  one (``flush(full=True)``: the whole string);
* TTL: the device copy is cleared when the mirrored EXPIRE deadline passes,
  as the Redis key would have vanished (README.md usage, ruby.rb:62).

Strings beyond one request: every write is cut into SETRANGE calls of at most
``chunk_bytes`` (default 8 MiB) and a key longer than that is read back with
GETRANGE chunks, so a multi-GB filter moves through a server whose
``proto-max-bulk-len`` admits the whole string without any one huge request
(stock Redis caps strings at 512 MB and raises for larger offsets, as SETBIT
would).

Extra options (all optional): ``device`` (HIP ordinal, default current),
``devices`` (a list of ordinals, or a count: one filter over several GPUs) with
``mode`` ``'replicated'`` (default) or ``'partitioned'`` (include/bfhip.h,
bf_config.devices), ``sync``, ``batch_keys`` / ``batch_bytes`` (host staging chunk
sizes), ``chunk_bytes`` (Redis request size).
"""
from __future__ import annotations

import time
from typing import Iterable, Optional

import numpy as np

from .. import keys as _keys
from .._lib import ArgumentError, BF_IMPORT_REPLACE, DIRTY_BLOCK_BYTES, Filter


class Hip:
    SYNC_MODES = ("write_through", "manual")

    def __init__(self, options: dict):
        self.options = options
        m, k = options.get("bits"), options.get("hashes")
        if m is None or k is None:
            raise ArgumentError("options[:bits] and options[:hashes] are required")
        if m <= 0:
            # the ruby driver would raise ZeroDivisionError / a Redis error at the first insert
            raise ArgumentError("filter size in bits must be positive (got %r)" % (m,))
        self.sync_mode = options.get("sync", "write_through")
        if self.sync_mode not in self.SYNC_MODES:
            raise ArgumentError("sync must be one of %s" % (self.SYNC_MODES,))
        self._clock = options.get("clock", time.monotonic)
        devices = options.get("devices")
        if isinstance(devices, int):   # `devices: 8` -> the first 8 GPUs
            devices = list(range(devices))
        flags = self._filter_flags()
        self.filter = Filter(m, k, device=options.get("device", -1),
                             batch_keys=options.get("batch_keys", 0),
                             batch_bytes=options.get("batch_bytes", 0),
                             flags=flags,
                             devices=devices, mode=str(options.get("mode", "replicated")))
        self.filter.track_dirty(True)
        # small write-through inserts replay their SETBITs (bf_insert_many_changes): whole-filter
        # (single-device) handles
        self._changes_ok = not devices
        self.chunk_bytes = int(options.get("chunk_bytes", 8 << 20))
        if self.chunk_bytes <= 0:
            raise ArgumentError("chunk_bytes must be positive")
        self._redis = None
        self._deadline: Optional[float] = None

    def _filter_flags(self) -> int:
        """bf_config.flags of the device filter (HipTest picks a hash engine here)."""
        return 0

    # -- attr_accessor :redis (ruby.rb:9); attaching imports the existing key
    @property
    def redis(self):
        return self._redis

    @redis.setter
    def redis(self, r):
        self._redis = r
        if r is not None:
            self.reload()

    @property
    def key_name(self) -> str:
        return self.options["key_name"]

    # -- TTL mirror.  The local deadline is taken on our clock BEFORE the EXPIRE / PTTL
    # request, so it never falls after the server's; when it passes, the device copy is
    # cleared and (write-through) the key is DELeted, so device and Redis agree from then
    # on instead of drifting apart by the TTL's rounding (the key was due to vanish
    # within one round trip anyway).
    def _expired(self) -> None:
        if self._deadline is not None and self._clock() >= self._deadline:
            self._deadline = None
            self.filter.clear()
            if self._redis is not None and self.sync_mode == "write_through":
                self._redis.delete(self.key_name)

    def _arm(self, expire) -> None:
        t0 = self._clock()
        self._deadline = t0 + float(expire)
        if self._redis is not None and self.sync_mode == "write_through":
            self._redis.expire(self.key_name, expire)

    # -- ruby.rb:15-17 / 57-63
    def insert(self, data, expire=None):
        return self.insert_many([data], expire)

    def insert_many(self, keys: Iterable, expire=None) -> bool:
        """Insert a batch; returns True iff some bit flipped (the ruby driver's !found)."""
        self._expired()
        buf, offs = _keys.pack(keys)
        # ruby.rb:62 `if !found && expire`: any expire but nil/false counts, 0 included
        armed = expire is not None and expire is not False
        write = self._redis is not None and self.sync_mode == "write_through"
        if write and self._changes_ok and self._setbit_sync(offs):
            # replay the SETBITs that changed something (ruby.rb:58-60) rather than SETRANGE whole
            # 64 KiB blocks: fewer bytes and Redis work whenever the batch flips fewer bits than
            # _setbit_sync's budget, and a concurrent writer's bits in those blocks are never
            # overwritten
            flips = self._insert_changes(buf, offs)
            if flips is not None:
                any_new = len(flips) > 0
                if any_new:
                    self._setbits(flips)
                if any_new and armed:
                    self._arm(expire)
                return any_new
        want = armed or write
        any_new, _ = self.filter.insert_many(buf, offs, any_new=want)
        if any_new:
            if write:
                self.flush()
            if armed:
                self._arm(expire)
        return bool(any_new) if want else None

    # Redis-side cost model of the two write-through forms: a pipelined SETBIT costs the server
    # about as much as SETRANGEing ~1 KB (~1 us vs ~1 ns per byte), so replay the flipped bits
    # while the batch's probes (an upper bound on its flips) stay under 1/1024 of the bytes the
    # dirty-block flush would send, and always for per-key calls.
    SETBIT_BYTES = 1024

    def _setbit_sync(self, offs: np.ndarray) -> bool:
        probes = (len(offs) - 1) * self.filter.k
        if probes <= Filter.CHANGES_MAX_PROBES:
            return True
        blocks = -(-self.filter.device_bytes // DIRTY_BLOCK_BYTES)
        flush_bytes = min(probes, blocks) * DIRTY_BLOCK_BYTES
        return probes * self.SETBIT_BYTES <= flush_bytes

    def _insert_changes(self, buf: np.ndarray, offs: np.ndarray):
        """Insert in bf_insert_many_changes-sized pieces; the flipped bits of all of them, or None
        (nothing inserted) when a key alone exceeds a piece's byte limit."""
        n = len(offs) - 1
        per = max(1, Filter.CHANGES_MAX_PROBES // self.filter.k)
        o64 = offs.astype(np.int64)
        if n and int(np.max(np.diff(o64))) > Filter.CHANGES_MAX_BYTES:
            return None
        parts, i = [], 0
        while i < n:
            j = int(np.searchsorted(o64, o64[i] + Filter.CHANGES_MAX_BYTES, side="right")) - 1
            j = min(j, i + per, n)
            parts.append(self.filter.insert_many_changes(buf, offs[i:j + 1]))
            i = j
        return np.concatenate(parts) if parts else np.zeros(0, np.uint64)

    def _setbits(self, offsets: np.ndarray) -> None:
        """SETBIT key o 1 for every offset, pipelined when the client can (ruby.rb:58-60)."""
        name, r = self.key_name, self._redis
        pipe = getattr(r, "pipeline", None)
        if pipe is not None:
            p = pipe(transaction=False)
            for o in offsets.tolist():
                p.setbit(name, o, 1)
            p.execute()
        else:
            for o in offsets.tolist():
                r.setbit(name, o, 1)

    # -- ruby.rb:20-30
    def include(self, key) -> bool:
        return bool(self.include_many([key])[0])

    def include_many(self, keys: Iterable) -> np.ndarray:
        """Membership of every key, as a numpy bool array (Ruby: Array<bool>)."""
        self._expired()
        buf, offs = _keys.pack(keys)
        return self.filter.include_many(buf, offs).astype(bool)

    # -- ruby.rb:33-35
    def clear(self):
        self.filter.clear()
        self._deadline = None
        if self._redis is not None:
            self._redis.delete(self.key_name)

    # -- Redis sync
    def flush(self, full: bool = False) -> int:
        """Write the device filter's changes to Redis; returns the bytes sent.

        SETRANGE per changed range keeps the TTL and grows the key like SETBIT would
        (the ranges are clipped to the trimmed string).  ``full``: the whole string."""
        ranges, rlen = self.filter.dirty_ranges(clear=self._redis is not None)
        if self._redis is None:
            return 0
        if full:
            ranges = [(0, rlen)] if rlen else []
        sent = 0
        for off, n in ranges:
            for c in range(off, off + n, self.chunk_bytes):
                ln = min(self.chunk_bytes, off + n - c)
                self._redis.setrange(self.key_name, c, self.filter.export_range(c, ln))
                sent += ln
        return sent

    def reload(self) -> None:
        """Replace the device filter with the Redis key's current value."""
        if self._redis is None:
            return
        data = self._read_key()
        self._deadline = None
        if data is None:
            self.filter.clear()
            return
        self.filter.import_redis(bytes(data), BF_IMPORT_REPLACE)
        self.filter.dirty_ranges(clear=True)   # device == Redis now
        t0 = self._clock()
        if hasattr(self._redis, "pttl"):   # milliseconds: no whole-second rounding
            ttl = self._redis.pttl(self.key_name)
            ttl = ttl / 1000.0 if ttl is not None and ttl > 0 else -1
        else:
            ttl = self._redis.ttl(self.key_name) if hasattr(self._redis, "ttl") else -1
            ttl = ttl - 1 if ttl is not None and ttl > 0 else -1   # TTL rounds up
        if ttl is not None and ttl > 0:
            self._deadline = t0 + ttl

    def _read_key(self):
        """GET, or GETRANGE chunks for a key longer than ``chunk_bytes``."""
        n = self._redis.strlen(self.key_name) if hasattr(self._redis, "strlen") else 0
        if n <= self.chunk_bytes:
            return self._redis.get(self.key_name)
        buf = bytearray(n)
        for c in range(0, n, self.chunk_bytes):
            part = self._redis.getrange(self.key_name, c, min(c + self.chunk_bytes, n) - 1)
            buf[c:c + len(part)] = part
        return bytes(buf)

    def to_redis_string(self) -> bytes:
        return self.filter.export_redis()

    def close(self):
        self.filter.close()
