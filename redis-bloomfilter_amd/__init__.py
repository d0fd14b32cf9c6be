"""redis-bloomfilter_amd — MI355X Bloom-filter engine behind the ``Redis::Bloomfilter`` API.

Importable as ``redis_bloomfilter_amd`` via ``pkgload.load()`` (the directory
name carries a hyphen).  Layout:

* ``csrc/``      HIP kernels (gfx950) + the C ABI of include/bfhip.h -> ``lib/libbfhip.so``
* ``_lib.py``    ctypes binding of that ABI (no CPU fallback)
* ``bloomfilter.py``  mirror of lib/redis/bloomfilter.rb (facade, sizing, driver lookup)
* ``drivers/hip.py``  the ``hip`` driver (mirror of lib/bloomfilter_driver/ruby.rb's interface)
* ``drivers/hip_lua.py``  the ``hip-lua`` driver (the Lua driver's scalable layout, lua.rb)
* ``keys.py``    Ruby ``to_s`` key marshalling and packing
* ``fakeredis.py``  in-memory Redis string-command model (no redis-server in this image)
* ``distributed.py`` multi-GPU layer (replicated / partitioned filters over torch.distributed)
* ``ruby/``      the Ruby-side drop-in (FFI driver) a maintainer adds to the gem
"""
from ._lib import (ArgumentError, BF_IMPORT_OR, BF_IMPORT_REPLACE, BfHipError, BfHipUnavailable,  # noqa: F401
                   BF_FLAG_ENGINE_MD5, BF_FLAG_ENGINE_SHA1, DIRTY_BLOCK_BYTES, Filter, LuaFilter, version)
from .bloomfilter import Bloomfilter, DRIVERS, VERSION, driver_name, register_driver  # noqa: F401
from .drivers.hip import Hip  # noqa: F401
from .drivers.hip_lua import HipLua  # noqa: F401
from .drivers.hip_test import HipTest  # noqa: F401
from .fakeredis import FakeRedis  # noqa: F401
from . import keys  # noqa: F401
from . import distributed  # noqa: F401

register_driver(Hip)
register_driver(HipLua)
register_driver(HipTest)
