"""``fluid.dygraph.dygraph_to_static`` (reference: fluid/dygraph/dygraph_to_static): the
framework's dy2static transcriber (jit/dy2static.py)."""
from ...jit.dy2static import *  # noqa: F401,F403
from ...jit import dy2static as program_translator  # noqa: F401
from ...jit import dy2static as convert_operators  # noqa: F401
