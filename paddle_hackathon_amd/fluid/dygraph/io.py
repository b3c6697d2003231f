from ...jit import TranslatedLayer  # noqa: F401

__all__ = ["TranslatedLayer"]
