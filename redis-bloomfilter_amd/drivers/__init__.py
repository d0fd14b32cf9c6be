"""Driver plugins (the ``Redis::BloomfilterDriver`` namespace)."""
from .hip import Hip
from .hip_lua import HipLua

__all__ = ["Hip", "HipLua"]
