"""``fluid.incubate.checkpoint.auto_checkpoint`` (reference: python/paddle/fluid/incubate/
checkpoint/auto_checkpoint.py: ``train_epoch_range`` and the checker)."""
from ....incubate.checkpoint import (train_epoch_range, register, AutoCheckpointChecker,  # noqa: F401
                                     latest_checkpoint)

__all__ = ["train_epoch_range", "register", "AutoCheckpointChecker", "latest_checkpoint"]
