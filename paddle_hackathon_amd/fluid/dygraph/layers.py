from ...nn.layer.layers import Layer  # noqa: F401

__all__ = ["Layer"]
