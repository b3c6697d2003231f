"""``incubate.nn.layer.fused_transformer`` (the fused layers of paddle.incubate.nn)."""
from ... import nn as _nn
from ...nn import *  # noqa: F401,F403
