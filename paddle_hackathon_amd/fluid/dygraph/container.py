from ...nn import Sequential, ParameterList, LayerList  # noqa: F401

__all__ = ["Sequential", "ParameterList", "LayerList"]
