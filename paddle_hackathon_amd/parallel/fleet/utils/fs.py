"""fleet.utils.fs (reference: python/paddle/distributed/fleet/utils/fs.py)."""
from . import LocalFS, HDFSClient  # noqa: F401

__all__ = ["LocalFS", "HDFSClient"]
