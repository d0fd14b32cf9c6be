"""``Redis::BloomfilterDriver::HipTest`` — the RubyTest driver's hash engines on the GPU.

lib/bloomfilter_driver/ruby_test.rb is the reference's benchmarking driver: the same Redis
bitstring and SETBIT/GETBIT semantics as ruby.rb, but probe i of a key is
``Digest::<E>.hexdigest("#{i}-#{key.to_s}").to_i(16) % bits`` (:43-61) with E picked by
``options[:hash_engine]`` (facade default ``'md5'``, bloomfilter.rb:15).  ``driver:
'hip-test'`` runs those engines in ``bf_engines.hip`` (``BF_FLAG_ENGINE_MD5`` /
``BF_FLAG_ENGINE_SHA1``) and keeps everything else of the ``hip`` driver: write-through
sync, dirty-block flushes, chunked transport, the TTL mirror.

``'crc32'`` is broken upstream (``Zlib.crc32(..)`` is an Integer and ``Integer#to_i``
takes no radix, :52), so, as there, the driver builds but every insert / include?
raises ``ArgumentError``; an unknown engine raises ``NameError`` (Ruby's NoMethodError
from ``send("engine_#{engine}")``, :46).  Per-key "was new" flags are not offered
(RubyTest#set returns nothing, :63-68).
"""
from __future__ import annotations

from typing import Iterable

from .._lib import ArgumentError, BF_FLAG_ENGINE_MD5, BF_FLAG_ENGINE_SHA1
from .hip import Hip


class HipTest(Hip):
    ENGINES = {"md5": BF_FLAG_ENGINE_MD5, "sha1": BF_FLAG_ENGINE_SHA1}

    def _filter_flags(self) -> int:
        engine = str(self.options.get("hash_engine", "md5"))
        self.engine = engine
        self._engine_error = None
        if engine == "crc32":
            self._engine_error = ArgumentError("engine_crc32: wrong number of arguments (given 1, expected 0) "
                                               "-- Integer#to_i takes no radix (ruby_test.rb:52)")
        elif engine not in self.ENGINES:
            self._engine_error = NameError("undefined method `engine_%s' for Redis::BloomfilterDriver::HipTest"
                                           % engine)
        return self.ENGINES.get(engine, BF_FLAG_ENGINE_MD5)

    def _check_engine(self) -> None:
        if self._engine_error is not None:
            raise self._engine_error

    def insert_many(self, keys: Iterable, expire=None):
        self._check_engine()
        return super().insert_many(keys, expire)

    def include_many(self, keys: Iterable):
        self._check_engine()
        return super().include_many(keys)
