"""Driver plugins (the ``Redis::BloomfilterDriver`` namespace)."""
from .hip import Hip

__all__ = ["Hip"]
