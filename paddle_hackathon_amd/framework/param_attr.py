"""ParamAttr (reference: python/paddle/fluid/param_attr.py)."""
from __future__ import annotations

__all__ = ["ParamAttr", "WeightNormParamAttr"]


class ParamAttr:
    def __init__(self, name=None, initializer=None, learning_rate=1.0, regularizer=None,
                 trainable=True, do_model_average=True, need_clip=True):
        self.name = name
        self.initializer = initializer
        self.learning_rate = learning_rate
        self.regularizer = regularizer
        self.trainable = trainable
        self.do_model_average = do_model_average
        self.need_clip = need_clip

    @staticmethod
    def _to_attr(arg):
        if arg is None:
            return ParamAttr()
        if isinstance(arg, ParamAttr):
            return arg
        if isinstance(arg, str):
            return ParamAttr(name=arg)
        if isinstance(arg, bool):
            return ParamAttr() if arg else False
        from ..nn.initializer import Initializer
        if isinstance(arg, Initializer):
            return ParamAttr(initializer=arg)
        from ..regularizer import WeightDecayRegularizer
        if isinstance(arg, WeightDecayRegularizer):
            return ParamAttr(regularizer=arg)
        raise TypeError(f"{type(arg)} cast to ParamAttr")


class WeightNormParamAttr(ParamAttr):
    def __init__(self, dim=None, **kwargs):
        super().__init__(**kwargs)
        self.dim = dim
