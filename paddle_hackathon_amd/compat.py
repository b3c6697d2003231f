"""Py2/3 compat helpers (reference: python/paddle/compat.py)."""
import math

__all__ = []

int_type = int
long_type = int


def to_text(obj, encoding="utf-8", inplace=False):
    if obj is None:
        return obj
    if isinstance(obj, list):
        out = [to_text(o, encoding) for o in obj]
        if inplace:
            obj[:] = out
            return obj
        return out
    if isinstance(obj, set):
        return {to_text(o, encoding) for o in obj}
    if isinstance(obj, dict):
        return {to_text(k, encoding): to_text(v, encoding) for k, v in obj.items()}
    return obj.decode(encoding) if isinstance(obj, bytes) else obj


def to_bytes(obj, encoding="utf-8", inplace=False):
    if obj is None:
        return obj
    if isinstance(obj, list):
        out = [to_bytes(o, encoding) for o in obj]
        if inplace:
            obj[:] = out
            return obj
        return out
    if isinstance(obj, set):
        return {to_bytes(o, encoding) for o in obj}
    return obj.encode(encoding) if isinstance(obj, str) else obj


def round(x, d=0):
    p = 10 ** d
    return float(math.floor((x * p) + math.copysign(0.5, x))) / p


def floor_division(x, y):
    return x // y


def get_exception_message(exc):
    return str(exc)
