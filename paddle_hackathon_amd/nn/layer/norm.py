"""``paddle.nn.layer.norm`` module path (reference: python/paddle/nn/layer/norm.py): the layers are in paddle.nn."""
from ...nn import *  # noqa: F401,F403
