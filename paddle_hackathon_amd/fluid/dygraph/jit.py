from ...jit import (TracedLayer, declarative, set_code_level, set_verbosity, save, load,  # noqa: F401
                    not_to_static, to_static)

dygraph_to_static_func = to_static

__all__ = ["TracedLayer", "declarative", "dygraph_to_static_func", "set_code_level", "set_verbosity", "save", "load",
           "not_to_static"]
