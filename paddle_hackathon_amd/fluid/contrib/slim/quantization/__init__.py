"""``fluid.contrib.slim.quantization`` (reference: python/paddle/fluid/contrib/slim/quantization):
static quantization passes, static post-training quantization and the dygraph QAT / PTQ tools.
The MKL-DNN int8 passes of the reference (quant_int8_mkldnn_pass, quant2_int8_mkldnn_pass) are
CPU-vendor specific and not part of an MI355X framework."""
from . import quantization_pass, post_training_quantization, imperative, cal_kl_threshold  # noqa: F401
from .quantization_pass import *  # noqa: F401,F403
from .post_training_quantization import *  # noqa: F401,F403
from .imperative import *  # noqa: F401,F403

__all__ = quantization_pass.__all__ + post_training_quantization.__all__ + imperative.__all__
