"""``paddle.incubate.passes`` (reference: python/paddle/incubate/passes/): program rewrites
registered with the pass manager (``paddle.distributed.passes.new_pass``)."""
from .fuse_resnet_unit_pass import fuse_resnet_unit  # noqa: F401

__all__ = ["fuse_resnet_unit"]
