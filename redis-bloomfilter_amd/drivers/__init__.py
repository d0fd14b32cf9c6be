"""Driver plugins (the ``Redis::BloomfilterDriver`` namespace)."""
from .hip import Hip
from .hip_lua import HipLua
from .hip_test import HipTest

__all__ = ["Hip", "HipLua", "HipTest"]
