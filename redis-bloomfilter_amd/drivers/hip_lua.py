"""``Redis::BloomfilterDriver::HipLua`` — the Lua driver's scalable filter on the GPU.

``driver: 'hip-lua'`` resolves here (``driver_name`` capitalises each dash-separated
part, bloomfilter.rb:77-79).  It keeps the Redis layout of lib/bloomfilter_driver/lua.rb
and vendor/assets/lua/add.lua / check.lua, so the Lua driver and this one read each
other's filters:

* ``KEYS[1]:count`` — the number of items that set a new bit (add.lua:5-11, 48-50);
* ``KEYS[1]:n``     — layer n's bitstring in SETBIT layout (add.lua:17, 38).

The layers live in HBM (``bf_lua*``, include/bfhip.h).  Attaching (``driver.redis =
r``) loads the count and every layer key; ``sync='write_through'`` (default) writes
the layers an insert touched back with SETRANGE and the count with SET, then EXPIREs
those layers when ``expire`` is given (add.lua:51-53); ``sync='manual'`` leaves Redis
alone until ``flush()``.
"""
from __future__ import annotations

import time
from typing import Dict, Iterable, List

import numpy as np

from .. import keys as _keys
from .._lib import ArgumentError, LuaFilter, lua_index


class HipLua:
    SYNC_MODES = ("write_through", "manual")

    def __init__(self, options: dict):
        self.options = options
        entries, precision = options.get("size"), options.get("error_rate")
        if entries is None or precision is None:
            raise ArgumentError("options[:size] and options[:error_rate] are required")
        self.sync_mode = options.get("sync", "write_through")
        if self.sync_mode not in self.SYNC_MODES:
            raise ArgumentError("sync must be one of %s" % (self.SYNC_MODES,))
        # ARGV[1], ARGV[2] reach Lua as strings and are read back as numbers (add.lua:1-2)
        self.entries, self.precision = float(entries), float(precision)
        self.filter = LuaFilter(self.entries, self.precision, device=options.get("device", -1))
        self._redis = None
        # TTL mirror per layer key (add.lua:51-53 EXPIREs the layer an item went into): the
        # deadline is taken before the EXPIRE request, so it never falls after the server's
        self._clock = options.get("clock", time.monotonic)
        self._deadlines: Dict[int, float] = {}

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

    CHANGES_MAX_KEYS = 64   # batches up to this many keys sync by SETBIT replay

    def _layer_key(self, n: int) -> str:
        return "%s:%d" % (self.key_name, n)

    # -- lua.rb:19-21 (add.lua)
    def insert(self, data, expire=None):
        return self.insert_many([data], expire)

    def _expired(self) -> None:
        """Layers whose mirrored TTL passed are gone in Redis: empty them on the device too
        (the count key has no TTL and stays, as in Redis)."""
        now = self._clock()
        for n in [n for n, t in self._deadlines.items() if now >= t]:
            del self._deadlines[n]
            self.filter.import_layer(n, b"")
            if self._redis is not None and self.sync_mode == "write_through":
                self._redis.delete(self._layer_key(n))

    def insert_many(self, keys: Iterable, expire=None) -> np.ndarray:
        """Insert in order, as one EVALSHA per key would; returns each key's INCR flag."""
        self._expired()
        buf, offs = _keys.pack(keys)
        write = self._redis is not None and self.sync_mode == "write_through"
        if write and len(offs) - 1 <= self.CHANGES_MAX_KEYS:
            # per-key (small) inserts replay the SETBITs that changed a layer (add.lua:43-47)
            # instead of SETRANGEing whole layer strings (a large filter's layer is 100s of MB)
            pk, touched, flips = self.filter.insert_many_changes(buf, offs)
            for layer, o in flips:
                self._redis.setbit(self._layer_key(layer), o, 1)
            if touched:
                self._redis.set("%s:count" % self.key_name, str(self.filter.count))
        else:
            pk, touched = self.filter.insert_many(buf, offs)
            if touched and write:
                self._write(touched)
        if touched and expire is not None and expire is not False:   # add.lua:51 tonumber(ARGV[4]): 0 is truthy
            t0 = self._clock()
            for n in touched:
                self._deadlines[n] = t0 + float(expire)
                if self._redis is not None and self.sync_mode == "write_through":
                    self._redis.expire(self._layer_key(n), expire)
        return pk.astype(bool)

    # -- lua.rb:23-26 (check.lua)
    def include(self, key) -> bool:
        return bool(self.include_many([key])[0])

    def include_many(self, keys: Iterable) -> np.ndarray:
        self._expired()
        buf, offs = _keys.pack(keys)
        return self.filter.include_many(buf, offs).astype(bool)

    # -- lua.rb:28-30
    def clear(self):
        self.filter.clear()
        self._deadlines.clear()
        if self._redis is not None:
            for k in self._redis.keys("%s:*" % self.key_name):
                self._redis.delete(k)

    # -- Redis sync
    def _write(self, layers: List[int]) -> None:
        for n in layers:
            data = self.filter.export_layer(n)
            if data:
                self._redis.setrange(self._layer_key(n), 0, data)
        self._redis.set("%s:count" % self.key_name, str(self.filter.count))

    def flush(self) -> None:
        """Write every layer and the count to Redis."""
        if self._redis is not None:
            self._write(list(range(1, self.filter.layers + 1)))

    def reload(self) -> None:
        """Replace the device layers with the Redis keys' values."""
        if self._redis is None:
            return
        self.filter.clear()
        self._deadlines.clear()
        raw = self._redis.get("%s:count" % self.key_name)
        count = int(raw) if raw is not None else 0
        self.filter.count = count
        if count:
            for n in range(1, lua_index(self.entries, count) + 1):
                t0 = self._clock()
                pttl = self._redis.pttl(self._layer_key(n)) if hasattr(self._redis, "pttl") else -1
                data = self._redis.get(self._layer_key(n))
                if data:
                    self.filter.import_layer(n, bytes(data))
                    if pttl is not None and pttl > 0:
                        self._deadlines[n] = t0 + pttl / 1000.0

    def close(self):
        self.filter.close()
