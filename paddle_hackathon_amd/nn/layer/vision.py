"""``paddle.nn.layer.vision`` module path (reference: python/paddle/nn/layer/vision.py): the layers are in paddle.nn."""
from ...nn import *  # noqa: F401,F403
