"""``distributed.passes.pass_base`` module path."""
from . import PassBase, PassContext, PassManager, PassType, new_pass, register_pass  # noqa: F401
