"""Dygraph quantization: QAT (ImperativeQuantAware) and PTQ (ImperativePTQ) — reference
fluid/contrib/slim/quantization/imperative/__init__.py."""
from . import qat, ptq, ptq_config, ptq_quantizer, ptq_registry  # noqa: F401
from .qat import *  # noqa: F401,F403
from .ptq import *  # noqa: F401,F403
from .ptq_config import *  # noqa: F401,F403
from .ptq_quantizer import *  # noqa: F401,F403
from .ptq_registry import *  # noqa: F401,F403

__all__ = qat.__all__ + ptq.__all__ + ptq_config.__all__ + ptq_quantizer.__all__ + ptq_registry.__all__
