"""``paddle.nn.layer.conv`` module path (reference: python/paddle/nn/layer/conv.py): the layers are in paddle.nn."""
from ...nn import *  # noqa: F401,F403
