"""``paddle.sysconfig`` (reference: python/paddle/sysconfig.py): header / library dirs for
building custom operators against this framework (HIP kernels link ``_C/libpha_kernels.so``)."""
import os

__all__ = ["get_include", "get_lib"]

_PKG = os.path.dirname(os.path.abspath(__file__))


def get_include():
    return os.path.join(_PKG, "csrc")


def get_lib():
    return os.path.join(_PKG, "_C")
