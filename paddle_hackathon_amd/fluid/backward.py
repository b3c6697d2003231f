from ..static.program import append_backward, gradients  # noqa: F401

__all__ = ["append_backward", "gradients"]
