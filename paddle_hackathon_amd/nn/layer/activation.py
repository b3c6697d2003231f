"""``paddle.nn.layer.activation`` module path (reference: python/paddle/nn/layer/activation.py): the layers are in paddle.nn."""
from ...nn import *  # noqa: F401,F403
