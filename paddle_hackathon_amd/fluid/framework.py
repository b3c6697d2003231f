"""``paddle.fluid.framework`` (reference: python/paddle/fluid/framework.py): Program / Variable /
guards / mode queries, on the framework's static Program IR (static/program.py)."""
from __future__ import annotations

import contextlib

from ..framework import core as _core
from ..framework.flags import set_flags, get_flags  # noqa: F401
from ..static.program import (Program, Variable, Block, OpDesc as Operator, default_main_program,  # noqa: F401
                              default_startup_program, program_guard, name_scope)
from ..static import cpu_places, cuda_places, xpu_places, mlu_places, npu_places, device_guard  # noqa: F401
from ..static import ipu_shard_guard, set_ipu_shard  # noqa: F401
from .core import is_compiled_with_cuda, is_compiled_with_rocm, is_compiled_with_xpu, is_compiled_with_npu  # noqa: F401

__all__ = ["Program", "default_startup_program", "default_main_program", "program_guard", "name_scope",
           "ipu_shard_guard", "set_ipu_shard", "cuda_places", "cpu_places", "xpu_places", "mlu_places",
           "cuda_pinned_places", "_non_static_mode", "in_dygraph_mode", "is_compiled_with_cinn",
           "is_compiled_with_cuda", "is_compiled_with_rocm", "is_compiled_with_xpu", "is_compiled_with_npu",
           "Variable", "require_version", "device_guard", "set_flags", "get_flags"]


def in_dygraph_mode():
    return _core.in_dynamic_mode()


_non_static_mode = in_dygraph_mode
_in_legacy_dygraph = in_dygraph_mode


def is_compiled_with_cinn():
    return False


def cuda_pinned_places(device_count=None):
    return [_core.CUDAPinnedPlace() for _ in range(device_count or 1)]


def require_version(min_version, max_version=None):
    """the MI355X build reports its own version; any requirement string parses and passes when the
    framework's version is within range"""
    from .. import __version__ as v

    def key(s):
        return tuple(int(p) for p in str(s).split(".")[:3] if p.isdigit())
    if key(v) and key(min_version) and key(v) < key(min_version) and key(v) != (0, 0, 0):
        raise Exception(f"version {v} < required {min_version}")
    return True


@contextlib.contextmanager
def _dygraph_guard(tracer=None):
    prev = _core._mode.static
    _core._mode.static = False
    try:
        yield
    finally:
        _core._mode.static = prev


def default_place():
    return _core.CUDAPlace(0) if _core._gpu_available() else _core.CPUPlace()


_current_expected_place = default_place

def switch_main_program(program):
    """make ``program`` the default main program; returns the previous one (reference:
    fluid/framework.py switch_main_program)"""
    from ..static import program as _P
    prev = _P._state.main
    _P._state.main = program
    return prev


def switch_startup_program(program):
    from ..static import program as _P
    prev = _P._state.startup
    _P._state.startup = program
    return prev


def __getattr__(name):   # ParamBase / EagerParamBase: the framework's Parameter
    if name in ("ParamBase", "EagerParamBase"):
        from ..framework.core import Parameter
        return Parameter
    raise AttributeError(name)
