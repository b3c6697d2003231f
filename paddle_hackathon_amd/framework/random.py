"""``paddle.framework.random`` (reference: python/paddle/framework/random.py)."""
from ..tensor.random import seed, get_cuda_rng_state, set_cuda_rng_state  # noqa: F401

__all__ = ["seed", "get_cuda_rng_state", "set_cuda_rng_state"]
