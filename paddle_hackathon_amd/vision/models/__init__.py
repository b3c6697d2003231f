"""``paddle.vision.models`` (reference: python/paddle/vision/models/__init__.py)."""
from .resnet import *  # noqa: F401,F403
from .zoo import *  # noqa: F401,F403
from . import resnet as _r, zoo as _z

__all__ = _r.__all__ + _z.__all__
