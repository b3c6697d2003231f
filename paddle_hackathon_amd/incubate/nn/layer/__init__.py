"""``incubate.nn.layer`` module paths (reference: python/paddle/incubate/nn/layer/)."""
from . import fused_transformer  # noqa: F401
