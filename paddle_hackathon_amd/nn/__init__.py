"""``paddle.nn`` (reference: python/paddle/nn/__init__.py)."""
from . import functional, initializer  # noqa: F401
from .layer.layers import Layer  # noqa: F401
from .layer.container import *  # noqa: F401,F403
from .layer.common import *  # noqa: F401,F403
from .layer.conv_norm_pool import *  # noqa: F401,F403
from .layer.loss import *  # noqa: F401,F403
from .layer.rnn import *  # noqa: F401,F403
from .layer.transformer import *  # noqa: F401,F403
from .clip import ClipGradByGlobalNorm, ClipGradByNorm, ClipGradByValue  # noqa: F401
from .decode import BeamSearchDecoder, dynamic_decode  # noqa: F401
from . import utils  # noqa: F401
from ..framework.core import Parameter  # noqa: F401
from ..framework.param_attr import ParamAttr  # noqa: F401

from .layer import container as _c, common as _cm, conv_norm_pool as _cn, loss as _l, rnn as _r, transformer as _t

__all__ = (["Layer", "ClipGradByGlobalNorm", "ClipGradByNorm", "ClipGradByValue", "BeamSearchDecoder",
            "dynamic_decode"] + _c.__all__ + _cm.__all__ + _cn.__all__ + _l.__all__ + _r.__all__ + _t.__all__)
from . import quant  # noqa: F401,E402

from . import loss  # noqa: E402,F401  (the paddle.nn.loss module path)
