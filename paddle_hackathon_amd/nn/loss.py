"""``paddle.nn.loss`` module path (the loss layers of nn/layer/loss.py)."""
from .layer.loss import *  # noqa: F401,F403
