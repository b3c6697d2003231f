"""``paddle.callbacks`` (reference: python/paddle/callbacks.py): the hapi callbacks."""
from .hapi.callbacks import *  # noqa: F401,F403
from .hapi.callbacks import __all__  # noqa: F401
