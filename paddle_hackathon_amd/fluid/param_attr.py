from ..framework.param_attr import ParamAttr, WeightNormParamAttr  # noqa: F401

__all__ = ["ParamAttr", "WeightNormParamAttr"]
