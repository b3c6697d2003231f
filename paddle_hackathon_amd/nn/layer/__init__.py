


def __getattr__(name):   # every paddle.nn layer under paddle.nn.layer (reference nn/layer/__init__.py)
    from ... import nn as _nn
    if name != "__path__" and hasattr(_nn, name):
        return getattr(_nn, name)
    raise AttributeError(name)
