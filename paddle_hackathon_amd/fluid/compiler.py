from ..static.program import CompiledProgram, BuildStrategy, ExecutionStrategy  # noqa: F401
from ..static import IpuCompiledProgram, IpuStrategy  # noqa: F401

__all__ = ["CompiledProgram", "ExecutionStrategy", "BuildStrategy", "IpuCompiledProgram", "IpuStrategy"]
