"""``paddle.fluid.unique_name`` (reference: python/paddle/fluid/unique_name.py)."""
from ..utils import unique_name as _un

generate = _un.generate
switch = _un.switch
guard = _un.guard

__all__ = ["generate", "switch", "guard"]
