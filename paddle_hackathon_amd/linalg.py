"""``paddle.linalg`` (reference: python/paddle/linalg.py) — re-exports tensor.linalg."""
from .tensor.linalg import (cholesky, norm, cond, cov, corrcoef, inv, eig, eigvals, multi_dot,  # noqa: F401
                            matrix_rank, svd, qr, lu, lu_unpack, matrix_power, det, slogdet, eigh, eigvalsh,
                            pinv, solve, cholesky_solve, triangular_solve, lstsq)

__all__ = ["cholesky", "norm", "cond", "cov", "corrcoef", "inv", "eig", "eigvals", "multi_dot", "matrix_rank",
           "svd", "qr", "lu", "lu_unpack", "matrix_power", "det", "slogdet", "eigh", "eigvalsh", "pinv", "solve",
           "cholesky_solve", "triangular_solve", "lstsq"]
