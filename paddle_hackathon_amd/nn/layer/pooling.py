"""``paddle.nn.layer.pooling`` module path (reference: python/paddle/nn/layer/pooling.py): the layers are in paddle.nn."""
from ...nn import *  # noqa: F401,F403
