"""Linear algebra (reference: python/paddle/tensor/linalg.py). Dense
factorizations run on rocSOLVER/MAGMA via PyTorch-ROCm."""
from __future__ import annotations

import torch

from ..framework.core import Tensor
from ..framework.dispatch import register_ops
from ._helpers import _u, _w, _axis
from .math import matmul, bmm, mv, dot  # noqa: F401
from .manipulation import transpose, t  # noqa: F401

__all__ = [
    "cholesky", "norm", "cond", "cov", "corrcoef", "inv", "inverse", "eig", "eigvals",
    "multi_dot", "matrix_rank", "svd", "qr", "lu", "lu_unpack", "matrix_power", "det",
    "slogdet", "eigh", "eigvalsh", "pinv", "solve", "cholesky_solve", "triangular_solve",
    "lstsq", "dist", "cross", "histogram", "bincount", "vector_norm", "matrix_norm",
]


def cholesky(x, upper=False, name=None):
    return _w(torch.linalg.cholesky(_u(x), upper=upper))


def norm(x, p="fro", axis=None, keepdim=False, name=None):
    tt = _u(x)
    d = _axis(axis)
    if p == "fro":
        if d is None:
            return _w(torch.linalg.vector_norm(tt, 2, keepdim=keepdim))
        return _w(torch.linalg.vector_norm(tt, 2, dim=d, keepdim=keepdim))
    if p == "nuc":
        return _w(torch.linalg.matrix_norm(tt, "nuc", dim=d if d is not None else (-2, -1), keepdim=keepdim))
    p = float(p)
    if d is None:
        return _w(torch.linalg.vector_norm(tt.reshape(-1), p, keepdim=False).reshape([1] * tt.dim() if keepdim else []))
    return _w(torch.linalg.vector_norm(tt, p, dim=d, keepdim=keepdim))


def vector_norm(x, p=2.0, axis=None, keepdim=False, name=None):
    return _w(torch.linalg.vector_norm(_u(x), p, dim=_axis(axis), keepdim=keepdim))


def matrix_norm(x, p="fro", axis=[-2, -1], keepdim=False, name=None):
    return _w(torch.linalg.matrix_norm(_u(x), p, dim=tuple(axis), keepdim=keepdim))


def cond(x, p=None, name=None):
    return _w(torch.linalg.cond(_u(x), p))


def cov(x, rowvar=True, ddof=True, fweights=None, aweights=None, name=None):
    tt = _u(x)
    if not rowvar:
        tt = tt.t()
    return _w(torch.cov(tt, correction=int(ddof), fweights=_u(fweights), aweights=_u(aweights)))


def corrcoef(x, rowvar=True, name=None):
    tt = _u(x)
    if not rowvar:
        tt = tt.t()
    return _w(torch.corrcoef(tt))


def inv(x, name=None):
    return _w(torch.linalg.inv(_u(x)))


inverse = inv


def eig(x, name=None):
    w, v = torch.linalg.eig(_u(x))
    return _w(w), _w(v)


def eigvals(x, name=None):
    return _w(torch.linalg.eigvals(_u(x)))


def eigh(x, UPLO="L", name=None):
    w, v = torch.linalg.eigh(_u(x), UPLO=UPLO)
    return _w(w), _w(v)


def eigvalsh(x, UPLO="L", name=None):
    return _w(torch.linalg.eigvalsh(_u(x), UPLO=UPLO))


def multi_dot(x, name=None):
    return _w(torch.linalg.multi_dot([_u(v) for v in x]))


def matrix_rank(x, tol=None, hermitian=False, name=None):
    return _w(torch.linalg.matrix_rank(_u(x), atol=_u(tol), hermitian=hermitian))


def svd(x, full_matrices=False, name=None):
    u, s, vh = torch.linalg.svd(_u(x), full_matrices=full_matrices)
    return _w(u), _w(s), _w(vh)


def qr(x, mode="reduced", name=None):
    q, r = torch.linalg.qr(_u(x), mode=mode)
    if mode == "r":
        return _w(r)
    return _w(q), _w(r)


def lu(x, pivot=True, get_infos=False, name=None):
    lu_, piv, info = torch.linalg.lu_factor_ex(_u(x), pivot=pivot)
    if get_infos:
        return _w(lu_), _w(piv.int()), _w(info.int())
    return _w(lu_), _w(piv.int())


def lu_unpack(x, y, unpack_ludata=True, unpack_pivots=True, name=None):
    p, l, u = torch.lu_unpack(_u(x), _u(y))
    return _w(p), _w(l), _w(u)


def matrix_power(x, n, name=None):
    return _w(torch.linalg.matrix_power(_u(x), n))


def det(x, name=None):
    return _w(torch.linalg.det(_u(x)))


def slogdet(x, name=None):
    s, l = torch.linalg.slogdet(_u(x))
    return _w(torch.stack([s, l]))


def pinv(x, rcond=1e-15, hermitian=False, name=None):
    return _w(torch.linalg.pinv(_u(x), rtol=rcond, hermitian=hermitian))


def solve(x, y, name=None):
    return _w(torch.linalg.solve(_u(x), _u(y)))


def cholesky_solve(x, y, upper=False, name=None):
    return _w(torch.cholesky_solve(_u(x), _u(y), upper=upper))


def triangular_solve(x, y, upper=True, transpose=False, unitriangular=False, name=None):
    a = _u(x)
    if transpose:
        a = a.transpose(-1, -2)
        upper = not upper
    return _w(torch.linalg.solve_triangular(a, _u(y), upper=upper, unitriangular=unitriangular))


def lstsq(x, y, rcond=None, driver=None, name=None):
    r = torch.linalg.lstsq(_u(x), _u(y), rcond=rcond, driver=driver)
    return _w(r.solution), _w(r.residuals), _w(r.rank), _w(r.singular_values)


def dist(x, y, p=2, name=None):
    return _w(torch.dist(_u(x), _u(y), p))


def cross(x, y, axis=9, name=None):
    a = _u(x)
    if axis == 9:
        axis = next(i for i, s in enumerate(a.shape) if s == 3)
    return _w(torch.linalg.cross(a, _u(y), dim=axis))


def histogram(input, bins=100, min=0, max=0, name=None):
    tt = _u(input).float()
    if min == 0 and max == 0:
        min, max = tt.min().item(), tt.max().item()
    return _w(torch.histc(tt, bins, min, max).long())


def bincount(x, weights=None, minlength=0, name=None):
    return _w(torch.bincount(_u(x), _u(weights), minlength))


register_ops(globals(), [n for n in __all__ if n not in ("transpose", "t")])
