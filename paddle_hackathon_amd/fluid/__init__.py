"""``paddle.fluid`` — the 1.x API of the reference (python/paddle/fluid/__init__.py) on the
MI355X framework: ``fluid.layers`` (1.x layer functions and control flow, LoD sequence ops over
padded kernels), ``fluid.dygraph`` (guard / to_variable / 1.x Layers), ``fluid.io``
(save/load_inference_model, save/load_params/persistables), ``fluid.core`` (LoDTensor, Scope,
places), ``Executor`` / ``Program`` / ``program_guard``, the 1.x optimizers, initializers,
regularizers, clips, metrics and nets."""
from __future__ import annotations

from . import core, framework, executor, layers, dygraph, io, initializer, param_attr, optimizer, regularizer, \
    clip, backward, unique_name, compiler, data_feeder, lod_tensor, metrics, nets, profiler, average, evaluator, \
    input, reader, contrib, transpiler, incubate, parallel_executor, device_worker, trainer_desc, \
    trainer_factory  # noqa: F401
from .framework import *  # noqa: F401,F403
from .executor import *  # noqa: F401,F403
from .data import data  # noqa: F401
from .initializer import set_global_initializer  # noqa: F401
from .backward import gradients, append_backward  # noqa: F401
from .input import embedding, one_hot  # noqa: F401
from .param_attr import ParamAttr, WeightNormParamAttr  # noqa: F401
from .data_feeder import DataFeeder  # noqa: F401
from .core import LoDTensor, LoDTensorArray, Scope, _Scope, CPUPlace, XPUPlace, CUDAPlace, CUDAPinnedPlace, \
    NPUPlace, IPUPlace, MLUPlace, CustomPlace  # noqa: F401
from .core import _cuda_synchronize  # noqa: F401
from .lod_tensor import create_lod_tensor, create_random_int_lodtensor  # noqa: F401
from .compiler import *  # noqa: F401,F403
from .parallel_executor import ParallelExecutor  # noqa: F401
from .dygraph.nn import *  # noqa: F401,F403
from .dygraph.layers import *  # noqa: F401,F403
from .dygraph.base import enable_dygraph, disable_dygraph  # noqa: F401
from .io import save, load, load_program_state, set_program_state  # noqa: F401
from .dygraph.checkpoint import save_dygraph, load_dygraph  # noqa: F401
from .transpiler import DistributeTranspiler, DistributeTranspilerConfig, HashName, RoundRobin  # noqa: F401
from .incubate import fleet  # noqa: F401
from ..framework.core import Tensor  # noqa: F401

enable_imperative = enable_dygraph
disable_imperative = disable_dygraph


class _InstallCheck:
    @staticmethod
    def run_check():
        from .. import utils
        return utils.run_check() if hasattr(utils, "run_check") else None


install_check = _InstallCheck()

__all__ = framework.__all__ + executor.__all__ + lod_tensor.__all__ + compiler.__all__ + backward.__all__ + [
    "io", "initializer", "embedding", "one_hot", "layers", "contrib", "data", "dygraph", "enable_dygraph",
    "disable_dygraph", "enable_imperative", "disable_imperative", "transpiler", "nets", "optimizer", "backward",
    "regularizer", "LoDTensor", "LoDTensorArray", "CPUPlace", "XPUPlace", "CUDAPlace", "CUDAPinnedPlace", "NPUPlace",
    "IPUPlace", "MLUPlace", "Tensor", "ParamAttr", "WeightNormParamAttr", "DataFeeder", "clip", "profiler",
    "unique_name", "Scope", "install_check", "save", "load", "_cuda_synchronize", "ParallelExecutor",
    "DistributeTranspiler", "DistributeTranspilerConfig", "HashName", "RoundRobin"]
