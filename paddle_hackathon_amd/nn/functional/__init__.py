"""``paddle.nn.functional`` (reference: python/paddle/nn/functional/__init__.py)."""
from .activation import *  # noqa: F401,F403
from .common import *  # noqa: F401,F403
from .conv import *  # noqa: F401,F403
from .pooling import *  # noqa: F401,F403
from .norm import *  # noqa: F401,F403
from .norm import batch_norm_act  # noqa: F401,E402
from .loss import *  # noqa: F401,F403
from .attention import *  # noqa: F401,F403
from .vision_ops import *  # noqa: F401,F403
from . import activation, common, conv, pooling, norm, loss, attention, vision_ops  # noqa: F401

__all__ = (activation.__all__ + common.__all__ + conv.__all__ + pooling.__all__ + norm.__all__
           + loss.__all__ + attention.__all__ + vision_ops.__all__)
