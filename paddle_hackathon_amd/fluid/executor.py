"""``paddle.fluid.executor`` (reference: python/paddle/fluid/executor.py)."""
from ..static.program import Executor, global_scope, scope_guard  # noqa: F401
from ..static.trainer import FetchHandler  # noqa: F401

__all__ = ["Executor", "global_scope", "scope_guard"]
