from .metrics import ChunkEvaluator, EditDistance, DetectionMAP  # noqa: F401

__all__ = ["ChunkEvaluator", "EditDistance", "DetectionMAP"]
