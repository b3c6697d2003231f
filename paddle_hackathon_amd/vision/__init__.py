"""``paddle.vision`` (reference: python/paddle/vision/__init__.py)."""
from . import models, transforms, datasets, ops  # noqa: F401
from .models import *  # noqa: F401,F403
from .transforms import *  # noqa: F401,F403
from .datasets import *  # noqa: F401,F403

_image_backend = "pil"


def set_image_backend(backend):
    global _image_backend
    if backend not in ("pil", "cv2", "tensor"):
        raise ValueError(backend)
    _image_backend = backend


def get_image_backend():
    return _image_backend


def image_load(path, backend=None):
    from PIL import Image
    return Image.open(path)


__all__ = ["set_image_backend", "get_image_backend", "image_load"]
