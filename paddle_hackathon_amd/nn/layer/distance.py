"""``paddle.nn.layer.distance`` module path (reference: python/paddle/nn/layer/distance.py): the layers are in paddle.nn."""
from ...nn import *  # noqa: F401,F403
