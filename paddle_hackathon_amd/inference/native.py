"""Python handle on the native inference engine (``_C/libpha_infer.so``, csrc/infer): a predictor
that runs a saved ``.pdmodel`` / ``.pdiparams`` pair with the C++ graph walker and the library's own
HIP kernels — no torch in the loop. Mirrors what a C / C++ service gets through ``pha_infer.h``
(the ``pha_infer_*`` handle API and the reference's ``PD_*`` C API subset).

Reference: paddle/fluid/inference/capi_exp/pd_predictor.h (PD_PredictorCreate / Run / handles)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_LIB = None
_DT = {np.dtype("float32"): 5, np.dtype("int64"): 3, np.dtype("int32"): 2}
_NP = {v: k for k, v in _DT.items()}


def lib_path():
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C", "libpha_infer.so")


def _lib():
    global _LIB
    if _LIB is None:
        path = lib_path()
        if not os.path.exists(path):
            from ..ops.build import build_infer
            build_infer()
        L = ctypes.CDLL(path)
        P, I, C = ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p
        L.pha_infer_create.argtypes = [C, C, I]
        L.pha_infer_create.restype = P
        L.pha_infer_create2.argtypes = [C, C, I, I]
        L.pha_infer_create2.restype = P
        L.pha_infer_create3.argtypes = [C, C, I, I, I]
        L.pha_infer_create3.restype = P
        L.pha_infer_applied_passes.argtypes = [P]
        L.pha_infer_applied_passes.restype = C
        L.pha_infer_pooled_bytes.argtypes = [P]
        L.pha_infer_pooled_bytes.restype = ctypes.c_size_t
        L.pha_infer_last_error.restype = C
        for f in ("pha_infer_num_inputs", "pha_infer_num_outputs"):
            getattr(L, f).argtypes = [P]
            getattr(L, f).restype = I
        for f in ("pha_infer_input_name", "pha_infer_output_name"):
            getattr(L, f).argtypes = [P, I]
            getattr(L, f).restype = C
        L.pha_infer_unsupported_ops.argtypes = [P]
        L.pha_infer_unsupported_ops.restype = C
        L.pha_infer_set_input.argtypes = [P, C, I, ctypes.POINTER(ctypes.c_int64), I, P]
        L.pha_infer_set_input.restype = I
        L.pha_infer_run.argtypes = [P]
        L.pha_infer_run.restype = I
        L.pha_infer_output_shape.argtypes = [P, I, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(I),
                                             ctypes.POINTER(I)]
        L.pha_infer_output_shape.restype = I
        L.pha_infer_copy_output.argtypes = [P, I, P, ctypes.c_size_t]
        L.pha_infer_copy_output.restype = I
        L.pha_infer_destroy.argtypes = [P]
        _LIB = L
    return _LIB


class NativePredictor:
    """``NativePredictor(model_file, params_file, device=-1, ir_optim=True)``: device -1 runs on the
    host, k >= 0 on GPU k (its own HIP stream and pooled device memory). ``run({name: ndarray})`` ->
    list of output ndarrays (fetch order). ``ir_optim`` folds conv + elementwise_add(bias) and conv +
    batch_norm at load (``applied_passes`` lists what fired). One predictor per thread (the
    reference PredictorPool model); the ctypes calls release the GIL. ``bf16`` (the reference's
    ``Config.enable_mkldnn_bfloat16``): on the GPU the matrix products (mul / matmul / fc and the
    im2col convolutions) run with bf16 operands on the kernel library's MFMA GEMM, fp32 elsewhere."""

    def __init__(self, model_file, params_file, device=-1, ir_optim=True, bf16=False):
        L = _lib()
        self._h = L.pha_infer_create3(model_file.encode(), (params_file or "").encode(), int(device),
                                      int(bool(ir_optim)), int(bool(bf16)))
        if not self._h:
            raise RuntimeError(f"native predictor: {L.pha_infer_last_error().decode()}")
        self.input_names = [L.pha_infer_input_name(self._h, i).decode() for i in range(L.pha_infer_num_inputs(self._h))]
        self.output_names = [L.pha_infer_output_name(self._h, i).decode()
                             for i in range(L.pha_infer_num_outputs(self._h))]
        self.unsupported = [s for s in L.pha_infer_unsupported_ops(self._h).decode().split(",") if s]
        self.applied_passes = [s for s in L.pha_infer_applied_passes(self._h).decode().split(";") if s]

    def pooled_bytes(self):
        """device bytes in this predictor's block pool"""
        return int(_lib().pha_infer_pooled_bytes(self._h))

    def run(self, feeds):
        L = _lib()
        for name, arr in feeds.items():
            a = np.ascontiguousarray(arr)
            if a.dtype not in _DT:
                a = a.astype(np.float32 if a.dtype.kind == "f" else np.int64)
            shape = (ctypes.c_int64 * max(a.ndim, 1))(*a.shape)
            if L.pha_infer_set_input(self._h, name.encode(), _DT[a.dtype], shape, a.ndim, a.ctypes.data) != 0:
                raise RuntimeError(L.pha_infer_last_error().decode())
        if L.pha_infer_run(self._h) != 0:
            raise RuntimeError(L.pha_infer_last_error().decode())
        outs = []
        for i in range(len(self.output_names)):
            shape = (ctypes.c_int64 * 8)()
            nd, dt = ctypes.c_int(), ctypes.c_int()
            if L.pha_infer_output_shape(self._h, i, shape, ctypes.byref(nd), ctypes.byref(dt)) != 0:
                raise RuntimeError(L.pha_infer_last_error().decode())
            out = np.empty([shape[k] for k in range(nd.value)], dtype=_NP[dt.value])
            if L.pha_infer_copy_output(self._h, i, out.ctypes.data, out.nbytes) != 0:
                raise RuntimeError(L.pha_infer_last_error().decode())
            outs.append(out)
        return outs

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _LIB is not None:
            _LIB.pha_infer_destroy(h)
            self._h = None
