"""Host-side mirror of ``Redis::Bloomfilter`` (lib/redis/bloomfilter.rb).

Same option names, defaults, sizing math, driver resolution and error
behaviour as the Ruby facade, so the parity tests read like the reference's
spec.  The reference's Ruby drop-in is ``ruby/lib/bloomfilter_driver/hip.rb``
(see INTEGRATION.md); this Python mirror is what the tests and the bench
drive, because there is no Ruby interpreter in this image.

Ruby ``include?`` is spelled ``include`` here (``?`` is not legal in a Python
identifier); the batched additions are ``insert_many`` / ``include_many``.
"""
from __future__ import annotations

import math
import re
from typing import Dict, Optional, Type

from . import fakeredis
from ._lib import ArgumentError

VERSION = "1.1.2"   # API level mirrored: lib/redis/bloomfilter/version.rb:5

# Redis::BloomfilterDriver namespace: CamelCase class name -> driver class.
DRIVERS: Dict[str, Type] = {}


def register_driver(cls: Type, name: Optional[str] = None) -> Type:
    DRIVERS[name or cls.__name__] = cls
    return cls


def _ruby_round(x: float) -> int:
    """Float#round: half away from zero; FloatDomainError on NaN/Infinity."""
    if math.isnan(x) or math.isinf(x):
        raise FloatingPointError("FloatDomainError: %r" % x)
    r = math.floor(abs(x) + 0.5)
    return int(r) if x >= 0 else -int(r)


def _ruby_log(x: float) -> float:
    """Math.log: log(0) is -Infinity; negative arguments raise Math::DomainError."""
    if x == 0:
        return -math.inf
    if x < 0:
        raise ValueError('Math::DomainError: Numerical argument is out of domain - "log"')
    return math.log(x)


def driver_name(driver: str) -> str:
    """bloomfilter.rb:77-79: ``'ruby-test'`` -> ``'RubyTest'``, ``'hip'`` -> ``'Hip'``."""
    parts = driver.lower().split("-")
    return "".join(re.sub(r"\w+", lambda m: m.group(0).capitalize(), t) for t in parts)


def _version_tuple(v: str):
    return tuple(int(x) for x in re.findall(r"\d+", v)[:3])


class Bloomfilter:
    """``Redis::Bloomfilter`` — bloomfilter.rb:3-81."""

    VERSION = VERSION

    @staticmethod
    def version() -> str:  # version.rb:6-8
        return "redis-bloomfilter version %s" % VERSION

    def __init__(self, options: Optional[dict] = None, **kw):
        caller = dict(options or {})
        caller.update(kw)
        # bloomfilter.rb:11-19 defaults (redis: Redis.current -> fakeredis.current()).
        self.options = {
            "size": 1000,
            "error_rate": 0.01,
            "key_name": "redis-bloomfilter",
            "hash_engine": "md5",
            "default_expire": None,
            "redis": None,
            "driver": None,
        }
        self.options.update(caller)
        # bloomfilter.rb:21 — checks the CALLER's hash, not the merged one.
        if caller.get("error_rate") is None or caller.get("size") is None:
            raise ArgumentError("options[:size] && options[:error_rate] cannot be nil")
        # bloomfilter.rb:25-28
        self.options["size"] = caller["size"]
        self.options["error_rate"] = caller["error_rate"]
        self.options["bits"] = Bloomfilter.optimal_m(caller["size"], self.options["error_rate"])
        self.options["hashes"] = Bloomfilter.optimal_k(caller["size"], self.options["bits"])

        self.redis = self.options["redis"] or fakeredis.current()   # :30
        if caller.get("hash_engine"):
            self.options["hash_engine"] = caller["hash_engine"]    # :31

        if self.options["driver"] is None:                          # :33-41
            ver = self.redis.info()["redis_version"]
            self.options["driver"] = "lua" if _version_tuple(ver) >= (2, 6, 0) else "ruby"

        name = driver_name(self.options["driver"])                  # :43 const_get
        if name not in DRIVERS:
            raise NameError("uninitialized constant Redis::BloomfilterDriver::%s" % name)
        self.driver = DRIVERS[name](self.options)
        self.driver.redis = self.redis                              # :45

    # bloomfilter.rb:50-52
    @staticmethod
    def optimal_m(num_of_elements, false_positive_rate=0.01) -> int:
        return _ruby_round((-1 * num_of_elements) * _ruby_log(false_positive_rate) / (math.log(2) ** 2))

    # bloomfilter.rb:54-58 (Integer division when both are Integers)
    @staticmethod
    def optimal_k(num_of_elements, bf_size) -> int:
        if isinstance(num_of_elements, int) and isinstance(bf_size, int):
            q = bf_size // num_of_elements
        else:
            q = bf_size / num_of_elements
        h = _ruby_round(math.log(2) * q)
        if h == 0:
            h += 1
        return h

    # bloomfilter.rb:61-73 (+ the batched delegators the hip driver adds)
    def _expire(self, expire):
        """``expire || @options[:default_expire]`` (bloomfilter.rb:62): only nil and false fall
        back to the default — 0 is truthy in Ruby and is passed on (EXPIRE key 0 deletes it)."""
        return self.options["default_expire"] if expire is None or expire is False else expire

    def insert(self, data, expire=None):
        return self.driver.insert(data, self._expire(expire))

    def include(self, key) -> bool:
        return self.driver.include(key)

    __contains__ = include

    def clear(self):
        return self.driver.clear()

    def insert_many(self, keys, expire=None):
        expire = self._expire(expire)
        if hasattr(self.driver, "insert_many"):
            return self.driver.insert_many(keys, expire)
        for k in keys:   # looping fallback for drivers without a batch path
            self.driver.insert(k, expire)
        return None

    def include_many(self, keys):
        if hasattr(self.driver, "include_many"):
            return self.driver.include_many(keys)
        return [self.driver.include(k) for k in keys]
