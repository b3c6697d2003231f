"""Transformer MLP  y = gelu_tanh(x W1 + b1) W2 + b2  as ONE autograd node with the GELU folded into
the GEMMs on either side of it.

Reference behaviour: ``fused_feedforward`` / the fused_gemm_epilogue op
(paddle/fluid/operators/fused/fused_gemm_epilogue_op.cu:29 bias+gelu forward with the
pre-activation kept as "reserve space", :298 dgelu + bias-grad backward), as used by the GPT
fleet models.

Three chains compute the same thing (a static choice, ``pick_mode``):

  0  fc1 GEMM (NT on the cached W1^T, ops/gemm.mm_nt) -> HIP bias+GELU pass; backward: NT dgrad
     of fc2 -> HIP dGELU+bias-grad pass
  1  own fc1 GEMM (ops/gemm.nn: transposed-store gemm4w) with bias + GELU + stored pre-activation
     in its epilogue; backward: own NT dgrad of fc2 with dGELU against the stored pre-activation
     and the fc1 bias-gradient column sums in its epilogue
  2  own fc1 GEMM (persistent gemm4p, NT) with bias + GELU + the stored pre-activation in its
     overlapped epilogue; backward as chain 0

Everything else (fc2 forward, both weight gradients, fc1 dgrad) runs on ops/gemm.py in both chains.
"""
from __future__ import annotations

import os

import torch

from . import gemm as G
from . import hip as _hip

def _eligible(x2d, w1, b1, w2, b2):
    return (x2d.is_cuda and x2d.dtype in (torch.bfloat16, torch.float16)
            and all(t is not None and t.dtype == x2d.dtype and t.is_contiguous() for t in (w1, b1, w2, b2))
            and w1.dim() == 2 and w2.dim() == 2 and w1.shape[1] == w2.shape[0] and x2d.shape[1] == w1.shape[0])


def _own_ok(x2d, w1, w2):
    M, H = x2d.shape
    F = w1.shape[1]
    return (G._own_ok("nn", x2d, w1, w2) and G.supported(F, M, H, w1, x2d) and G.supported(M, F, H, x2d, w2))


def _fwd(mode, x2d, w1, b1, approximate=True):
    """-> (activation, saved pre-activation); modes 0 / 2 save x W1 (bias not added), mode 1 x W1 + b1.
    approximate=False (exact erf GELU, BERT): mode 0 only (the GEMM epilogues compute tanh-GELU)"""
    if mode == 1:
        return G.nn(x2d, w1, bias=b1, act="gelu", aux_out=True)
    from .conv_gemm import weight_t
    if mode == 2:
        r = G.mm_nt_bias_gelu(x2d, weight_t(w1), b1)
        if r is not None:
            return r
    h = G.mm_nt(x2d, weight_t(w1))
    return _hip.bias_gelu_fwd(h, b1, approximate), h


def _bwd_gelu(mode, gy, w2, pre, b1, want_db=True, approximate=True):
    """-> (d pre-activation, d b1 or None with want_db=False) from the MLP output gradient"""
    if mode == 1:
        g, part = G.gemm(gy, w2, False, False, act="dgelu", aux=pre, colsum=True)
        return g, G.colsum_finish(part, b1.dtype)
    ga = G.mm_nt(gy, w2)
    return _hip.bias_gelu_bwd(ga, pre, b1, approximate, want_db=want_db)


_MODES = {"pass": 0, "force": 1, "epi": 2}


def pick_mode(x2d, w1, b1, w2):
    """static (the same on every rank): PHA_FUSED_MLP = "pass" (chain 0), "epi" (chain 2: fc1 on the
    persistent gemm4p with bias + GELU + pre-activation in its epilogue, backward as chain 0) or
    "force" (chain 1, the gemm4w fused chain, measured behind chain 0 in round 2:
    profiles/gpt3_mlp_chain_pick_ab_r2.log)"""
    mode = _MODES.get(os.environ.get("PHA_FUSED_MLP", _DEFAULT), 0)
    if mode == 1 and not _own_ok(x2d, w1, w2):
        return 0
    return mode


# chain 2 by default: fc1's bias + GELU live in the GEMM that produces them (882 vs 967 us per
# layer for library GEMM + pass, profiles/mlp_epi_ab_r3/gelu_epi.log; full GPT step within noise
# of chain 0 in an alternating A/B, ab_*.log)
_DEFAULT = "epi"


class FusedMLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, w1, b1, w2, b2, mode, approximate=True):
        from .conv_gemm import weight_t
        a, pre = _fwd(mode, x2d, w1, b1, approximate)
        y = G.mm_nt(a, weight_t(w2)) if b2 is None else G.mm_nt_bias(a, weight_t(w2), b2)
        ctx.save_for_backward(x2d, w1, b1, w2, pre, a)
        ctx.mode, ctx.approximate = mode, approximate
        return y

    @staticmethod
    def backward(ctx, gy):
        from .conv_gemm import weight_grad
        x2d, w1, b1, w2, pre, a = ctx.saved_tensors
        gy = gy.contiguous()
        # both bias gradients come out of the weight-gradient GEMMs that already read dY / dpre
        # (G.mm_tn_db: column sums of the TN kernel's B fragments), no separate pass over either
        if ctx.needs_input_grad[4]:
            dw2, db2 = G.mm_tn_db(a, gy)
        else:
            dw2, db2 = weight_grad(a, gy), None
        fused_db = ctx.mode != 1
        g, db1 = _bwd_gelu(ctx.mode, gy, w2, pre, b1, want_db=not fused_db, approximate=ctx.approximate)
        dx = G.mm_nt(g, w1) if ctx.needs_input_grad[0] else None
        if fused_db:
            dw1, db1 = G.mm_tn_db(x2d, g, b1.dtype)
        else:
            dw1 = weight_grad(x2d, g)
        return dx, dw1, db1, dw2, db2, None, None


def fused_mlp(x, w1, b1, w2, b2, approximate=True):
    """gelu(x @ w1 + b1) @ w2 + b2 for x [..., H], w1 [H, F], w2 [F, H] (Paddle [in, out]); tanh
    GELU by default, exact (erf) with approximate=False (chain 0: GEMM + bias-GELU pass);
    b2 None: no output bias (the caller adds it, e.g. in the next add-LN kernel)"""
    x2d = x.reshape(-1, x.shape[-1])
    if not x2d.is_contiguous():
        x2d = x2d.contiguous()
    mode = pick_mode(x2d, w1, b1, w2) if approximate else 0
    y = FusedMLP.apply(x2d, w1, b1, w2, b2, mode, bool(approximate))
    return y.reshape(list(x.shape[:-1]) + [w2.shape[1]])


def available(x, w1, b1, w2, b2):
    from . import fused
    return fused._use_hip(x) and _eligible(x.reshape(-1, x.shape[-1]), w1, b1, w2, b2) \
        and os.environ.get("PHA_LINEAR_NT", "1") != "0"
