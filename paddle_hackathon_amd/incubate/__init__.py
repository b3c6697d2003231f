"""``paddle.incubate`` (reference: python/paddle/incubate/__init__.py)."""
from __future__ import annotations

from .optimizer import LookAhead, ModelAverage, DistributedFusedLamb  # noqa: F401
from .operators import (graph_send_recv, graph_khop_sampler, graph_reindex, graph_sample_neighbors,  # noqa: F401
                        segment_sum, segment_mean, segment_max, segment_min, softmax_mask_fuse,
                        softmax_mask_fuse_upper_triangle, identity_loss)
from . import optimizer  # noqa: F401
from . import nn  # noqa: F401
from . import autograd  # noqa: F401
from . import asp  # noqa: F401
from . import checkpoint  # noqa: F401
from ..fluid.incubate.checkpoint import auto_checkpoint  # noqa: F401
from . import distributed  # noqa: F401
from . import autotune  # noqa: F401
from . import operators  # noqa: F401
from . import passes  # noqa: F401
from .passes import fuse_resnet_unit_pass  # noqa: F401
from ..fluid.layer_helper import LayerHelper  # noqa: F401
from .. import sparse  # noqa: F401

__all__ = ["LookAhead", "ModelAverage", "softmax_mask_fuse_upper_triangle", "softmax_mask_fuse", "graph_send_recv",
           "graph_khop_sampler", "graph_sample_neighbors", "graph_reindex", "segment_sum", "segment_mean",
           "segment_max", "segment_min", "identity_loss"]


def __getattr__(name):
    if name == "multiprocessing":
        import importlib
        return importlib.import_module(".multiprocessing", __name__)
    raise AttributeError(name)
