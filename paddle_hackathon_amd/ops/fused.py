"""Fused hot ops: HIP kernels on gfx950, PyTorch reference path on CPU.

Reference parity (what each op replaces in the reference):
  * layer_norm       — phi/kernels/gpu/layer_norm_kernel.cu, layer_norm_grad_kernel.cu
  * softmax          — phi/kernels/gpu/softmax_kernel.cu (gpudnn/softmax_gpudnn.h)
  * softmax_cross_entropy — phi/kernels/gpu/cross_entropy_kernel.cu (softmax_with_cross_entropy)
  * gelu / bias_gelu — phi/kernels/gpu/gelu_kernel.cu, operators/fused/fused_dropout_act_bias.h
  * fused_adam_      — phi/kernels/gpu/adam_kernel.cu (+ multi_tensor_adam in fluid/operators/optimizers)
  * fused_momentum_  — phi/kernels/gpu/merged_momentum_kernel.cu
  * flash_attention  — operators/fused/fused_attention_op.cu, fmha_ref.h
  * embedding        — phi/kernels/gpu/embedding_kernel.cu
  * bias_dropout_residual_layer_norm — operators/fused/fused_bias_dropout_residual_layer_norm_op.cu
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as TF

from . import _lib
from . import hip as _hip

_native = None


def _is_dtensor(t):
    from torch.distributed.tensor import DTensor
    return isinstance(t, DTensor)


def _use_hip(t: torch.Tensor) -> bool:
    global _native
    if not t.is_cuda or type(t) is not torch.Tensor and _is_dtensor(t):
        return False   # distributed tensors run on torch ops (sharding propagation), not raw pointers
    if _native is None:
        _native = _lib.require_native()
    return _native


# ----------------------------------------------------------------------------
# GELU / bias-GELU
# ----------------------------------------------------------------------------
class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, approximate):
        ctx.save_for_backward(x, b)
        ctx.approximate = approximate
        return _hip.bias_gelu_fwd(x, b, approximate)

    @staticmethod
    def backward(ctx, gy):
        x, b = ctx.saved_tensors
        gx, gb = _hip.bias_gelu_bwd(gy.contiguous(), x, b, ctx.approximate)
        return gx, gb, None


def gelu(x, approximate=False):
    if _use_hip(x) and x.dtype in (torch.bfloat16, torch.float32, torch.float16) and x.is_contiguous():
        return _BiasGelu.apply(x, None, bool(approximate))
    return TF.gelu(x, approximate="tanh" if approximate else "none")


def bias_gelu(x, b, approximate=False):
    """gelu(x + b) with b broadcast over the last dim."""
    if _use_hip(x) and x.dtype in (torch.bfloat16, torch.float32, torch.float16) and x.is_contiguous() and b.dim() == 1 and b.dtype == x.dtype:
        return _BiasGelu.apply(x, b, bool(approximate))
    return TF.gelu(x + b, approximate="tanh" if approximate else "none")


def add_relu(x, y):
    return torch.relu(x + y)


# ----------------------------------------------------------------------------
# softmax
# ----------------------------------------------------------------------------
class _Softmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = _hip.softmax_fwd(x)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        return _hip.softmax_bwd(gy.contiguous(), y)


def softmax(x, axis=-1):
    if axis in (-1, x.dim() - 1) and _use_hip(x) and x.dtype in (torch.bfloat16, torch.float32, torch.float16) and x.is_contiguous() and x.shape[-1] <= 16384:
        return _Softmax.apply(x)
    return torch.softmax(x, axis)


# ----------------------------------------------------------------------------
# LayerNorm / RMSNorm
# ----------------------------------------------------------------------------
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        y, mean, rstd = _hip.layer_norm_fwd(x, w, b, eps)
        ctx.save_for_backward(x, w, b, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, b, mean, rstd = ctx.saved_tensors
        gx, gw, gb = _hip.layer_norm_bwd(gy.contiguous(), x, w, mean, rstd, b is not None)
        return gx, gw, gb, None


def layer_norm(x, normalized_shape, weight=None, bias=None, eps=1e-5):
    H = 1
    for s in normalized_shape:
        H *= s
    if (_use_hip(x) and x.is_contiguous() and x.dtype in (torch.bfloat16, torch.float32, torch.float16)
            and weight is not None and weight.dtype in (x.dtype, torch.float32) and H % 8 == 0 and H <= 4096
            and (bias is None or bias.dtype == weight.dtype)):
        return _LayerNorm.apply(x, weight.reshape(-1), None if bias is None else bias.reshape(-1), float(eps))
    ns = list(normalized_shape)
    # torch's kernel wants one dtype: fp32 master LN weights (AMP O2) are cast to the input's
    return TF.layer_norm(x, ns, None if weight is None else weight.reshape(ns).to(x.dtype),
                         None if bias is None else bias.reshape(ns).to(x.dtype), eps)


class _AddLayerNorm(torch.autograd.Function):
    """(x, r) -> (h = x + r, y = LN(h)) in one kernel; backward folds dh into dx.
    With ``xb`` (the bias of the branch output r, e.g. an attention / MLP output projection run
    without its bias): h = x + (r + xb); the backward's LN kernel also sums dh over the rows,
    which is xb's gradient — no separate column-sum pass over dh in the projection's backward."""

    @staticmethod
    def forward(ctx, x, r, w, b, eps, xb=None):
        if xb is None:
            y, mean, rstd, h = _hip.layer_norm_fwd(x, w, b, eps, residual=r)
        else:
            y, mean, rstd, h = _hip.bdrln_fwd(r, xb, x, w, b, eps, 0, 0, 1.0)
        ctx.save_for_backward(h, w, b, mean, rstd)
        ctx.xb_dtype = None if xb is None else xb.dtype
        return h, y

    @staticmethod
    def backward(ctx, gh, gy):
        h, w, b, mean, rstd = ctx.saved_tensors
        xbd = ctx.xb_dtype
        if gy is None:
            gxb = None if xbd is None else gh.reshape(-1, gh.shape[-1]).sum(0, dtype=torch.float32).to(xbd)
            return gh, gh, None, None, None, gxb
        res = _hip.layer_norm_bwd(gy.contiguous(), h, w, mean, rstd, b is not None,
                                  dres=None if gh is None else gh.contiguous(), dx_colsum=xbd)
        gx, gw, gb = res[:3]
        gxb = None if xbd is None else (res[3] if res[3].dtype == xbd else res[3].to(xbd))
        return gx, gx, gw, gb, None, gxb


def add_layer_norm(x, residual, weight, bias=None, eps=1e-5, xb=None):
    """Pre-LN residual step: returns (h, LN(h)) with h = x + residual (one HIP kernel each way);
    ``xb`` (optional): a bias of ``residual`` added in the same pass (h = x + (residual + xb))."""
    H = weight.numel()
    if (_use_hip(x) and x.is_contiguous() and residual.is_contiguous() and residual.dtype == x.dtype
            and residual.shape == x.shape and x.dtype in (torch.bfloat16, torch.float32, torch.float16)
            and weight.dtype in (x.dtype, torch.float32) and H % 8 == 0 and H <= 4096
            and (bias is None or bias.dtype == weight.dtype) and (xb is None or xb.numel() == H)):
        return _AddLayerNorm.apply(x, residual, weight.reshape(-1), None if bias is None else bias.reshape(-1),
                                   float(eps), None if xb is None else xb.reshape(-1))
    h = x + (residual if xb is None else residual + xb)
    return h, layer_norm(h, [H], weight, bias, eps)


def rms_norm(x, weight, eps=1e-6):
    v = x.float().pow(2).mean(-1, keepdim=True)
    y = (x.float() * torch.rsqrt(v + eps)).to(x.dtype)
    return y * weight if weight is not None else y


# PHA_LN_DROP_FUSED=0: LN backward and the dropout backward as two passes (A/B switch)
_LN_DROP_FUSED = os.environ.get("PHA_LN_DROP_FUSED", "1") != "0"


class _BiasDropoutResidualLN(torch.autograd.Function):
    """y = LN(residual + dropout(x + bias)) in one HIP pass (hs stored for the backward); the dropout
    mask is a counter hash of (seed, element) regenerated in the backward, never stored.
    Backward: LN backward (d residual = dh) then one pass dx = dh * mask / (1-p) with the bias
    gradient as its column sums (reference fused_bias_dropout_residual_layer_norm_op.cu)."""

    @staticmethod
    def forward(ctx, x, residual, bias, w, b, p, eps):
        thresh = min(65535, int(round(p * 65536))) if p > 0 else 0
        kscale = 1.0 / (1.0 - p) if p > 0 else 1.0
        seed, seed_dev = _hip.dropout_seed(x.device) if thresh else (0, None)
        y, mean, rstd, hs = _hip.bdrln_fwd(x, bias, residual, w, b, eps, seed, thresh, kscale, seed_dev)
        ctx.save_for_backward(hs, w, mean, rstd)
        ctx.cfg = (seed, thresh, kscale, b is not None, None if bias is None else bias.dtype)
        ctx.seed_dev = seed_dev
        return y

    @staticmethod
    def backward(ctx, gy):
        hs, w, mean, rstd = ctx.saved_tensors
        seed, thresh, kscale, has_b, xb_dt = ctx.cfg
        if thresh and xb_dt is None and _LN_DROP_FUSED:   # one pass: LN backward + dropout'
            dh, dx, dw, db = _hip.layer_norm_dropout_bwd(gy.contiguous(), hs, w, mean, rstd, has_b, seed, thresh,
                                                         kscale, ctx.seed_dev)
            return dx, dh, None, dw, db, None, None
        dh, dw, db = _hip.layer_norm_bwd(gy.contiguous(), hs, w, mean, rstd, has_b)
        if thresh == 0 and xb_dt is None:
            dx, dxb = dh, None
        else:
            dx, dxb = _hip.dropout_bias_bwd(dh, seed, thresh, kscale, xb_dt, ctx.seed_dev)
        return dx, dh, dxb, dw, db, None, None


def bias_dropout_residual_layer_norm(x, residual, bias, ln_w, ln_b, dropout_p, training, eps):
    """LN(residual + dropout(x + bias)) over the last dim (reference incubate
    fused_bias_dropout_residual_layer_norm)."""
    p = float(dropout_p) if training else 0.0
    H = x.shape[-1]
    if (_use_hip(x) and x.is_contiguous() and residual.is_contiguous() and residual.shape == x.shape
            and residual.dtype == x.dtype and x.dtype in (torch.bfloat16, torch.float32, torch.float16)
            and ln_w is not None and ln_w.numel() == H and ln_w.dtype in (x.dtype, torch.float32)
            and (ln_b is None or ln_b.dtype == ln_w.dtype) and H % 8 == 0 and H <= 4096 and p < 1.0):
        return _BiasDropoutResidualLN.apply(x, residual, bias, ln_w.reshape(-1),
                                            None if ln_b is None else ln_b.reshape(-1), p, float(eps))
    h = x + bias if bias is not None else x
    if p > 0:
        h = TF.dropout(h, p, True)
    h = h + residual
    return layer_norm(h, [H], ln_w, ln_b, eps)


# ----------------------------------------------------------------------------
# softmax cross-entropy (hard labels)
# ----------------------------------------------------------------------------
class _SoftmaxCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        loss, lse = _hip.softmax_ce_fwd(logits, labels, ignore_index)
        ctx.save_for_backward(logits, labels, lse)
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, gloss):
        logits, labels, lse = ctx.saved_tensors
        gx = _hip.softmax_ce_bwd(gloss.contiguous().float(), logits, labels, lse, ctx.ignore_index)
        return gx, None, None


def softmax_cross_entropy(logits, labels, ignore_index=-100):
    """Per-row loss (fp32) of softmax CE with int labels; logits [..., V]."""
    shp = logits.shape[:-1]
    V = logits.shape[-1]
    l2 = logits.reshape(-1, V)
    lab = labels.reshape(-1)
    if _use_hip(logits) and logits.dtype in (torch.bfloat16, torch.float32, torch.float16) and V > 0:
        if not l2.is_contiguous():
            l2 = l2.contiguous()
        loss = _SoftmaxCE.apply(l2, lab.to(torch.int64).contiguous(), int(ignore_index))
    else:
        l2 = l2.float() if l2.dtype in (torch.float16, torch.bfloat16) else l2
        loss = TF.cross_entropy(l2, lab.long(), reduction="none", ignore_index=ignore_index)
    return loss.reshape(shp)


# ----------------------------------------------------------------------------
# embedding
# ----------------------------------------------------------------------------
class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, padding_idx):
        ctx.save_for_backward(ids)
        ctx.num = w.shape[0]
        ctx.padding_idx = padding_idx
        return _hip.embedding_fwd(ids, w)

    @staticmethod
    def backward(ctx, gy):
        (ids,) = ctx.saved_tensors
        if _hip.embedding_bwd_supported(gy, ids.numel()):
            return None, _hip.embedding_bwd(ids, gy, ctx.num, ctx.padding_idx), None
        from . import fallback
        fallback.note("embedding_grad", f"{gy.dtype} D={gy.shape[-1]} -> aten")
        gw = torch.ops.aten.embedding_dense_backward(gy, ids, ctx.num, ctx.padding_idx if ctx.padding_idx is not None else -1, False)
        return None, gw, None


def embedding(ids, weight, padding_idx=None, sparse=False):
    if _use_hip(weight) and weight.is_contiguous() and (weight.shape[1] * weight.element_size()) % 16 == 0 and weight.dtype in (torch.bfloat16, torch.float32, torch.float16):
        return _Embedding.apply(ids.contiguous(), weight, padding_idx)
    if weight.is_cuda:
        from . import fallback
        fallback.note("embedding", f"{weight.dtype} {tuple(weight.shape)} -> torch")
    return TF.embedding(ids, weight, padding_idx)


# ----------------------------------------------------------------------------
# attention
# ----------------------------------------------------------------------------
def flash_attention(q, k, v, causal=False, dropout_p=0.0, scale=None, training=True, mask=None):
    """q, k, v: [B, S, H, D] (Paddle's fused-attention layout). Returns [B, S, H, D].
    mask: additive float (or boolean keep-) mask broadcastable to [B, H, S, Sk]."""
    drop = dropout_p if training else 0.0
    if _use_hip(q) and _hip.flash_attn_supported(q, k, v, drop, mask):
        return _hip.flash_attention_any(q, k, v, causal, scale, mask, drop)
    if q.is_cuda:
        from . import fallback
        fallback.note("attention", f"{q.dtype} D={q.shape[-1]} mask={mask is not None} -> torch SDPA")
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    m = mask
    if m is not None and m.dtype != torch.bool:
        m = m.to(q.dtype)
    o = TF.scaled_dot_product_attention(qt, kt, vt, attn_mask=m, dropout_p=drop, is_causal=causal and m is None,
                                        scale=scale)
    return o.transpose(1, 2)


def flash_attention_qkvpacked(qkv, num_heads, causal=False, dropout_p=0.0, scale=None, training=True, mask=None):
    """qkv: [B, S, 3*H*D] or [B, S, H, 3D] fused projection (per head q|k|v) -> [B, S, H, D].
    With a mask or dropout the extension kernels write the packed gradient in place (no
    split-backward concatenation)."""
    B, S = qkv.shape[0], qkv.shape[1]
    q4 = qkv.reshape(B, S, num_heads, -1)
    drop = dropout_p if training else 0.0
    if (mask is not None or drop) and _use_hip(q4):
        o = _hip.flash_attention_packed_ext(q4, causal, scale, mask, drop)
        if o is not None:
            return o
    if (_use_hip(q4) and not (training and dropout_p > 0) and q4.is_contiguous()
            and (scale is None or scale > 0)   # the packed forward folds a positive scale into its max
            and _hip.flash_attn_packed_supported(q4, num_heads)):
        return _hip.FlashAttentionPacked.apply(q4, bool(causal), scale)
    D = q4.shape[-1] // 3
    q, k, v = q4.split(D, dim=-1)
    return flash_attention(q, k, v, causal=causal, dropout_p=dropout_p, scale=scale, training=training, mask=mask)


# ----------------------------------------------------------------------------
# optimizers / AMP helpers (multi-tensor)
# ----------------------------------------------------------------------------
def fused_adam_(params, grads, exp_avgs, exp_avg_sqs, masters, lr, beta1, beta2, eps, step,
                weight_decay=0.0, decoupled=True, lr_ratios=None, grad_scale=1.0):
    """In-place Adam/AdamW over lists. ``masters`` (fp32) may be None entries
    (params then fp32 themselves). ``step`` is the 1-based step count."""
    if params and _use_hip(params[0]):
        return _hip.multi_tensor_adam(params, grads, exp_avgs, exp_avg_sqs, masters, lr, beta1, beta2,
                                      eps, step, weight_decay, decoupled, lr_ratios, grad_scale)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    with torch.no_grad():
        for i, (p, g, m, v) in enumerate(zip(params, grads, exp_avgs, exp_avg_sqs)):
            if g is None:
                continue
            mp = masters[i] if masters is not None and masters[i] is not None else p
            lr_i = lr * (lr_ratios[i] if lr_ratios is not None else 1.0)
            gf = g.float() * grad_scale if grad_scale != 1.0 else g.float()
            if weight_decay and not decoupled:
                gf = gf + weight_decay * mp.float()
            m.mul_(beta1).add_(gf, alpha=1 - beta1)
            v.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
            upd = (m / bc1) / denom
            newp = mp.float()
            if weight_decay and decoupled:
                newp = newp * (1 - lr_i * weight_decay)
            newp = newp - lr_i * upd
            mp.copy_(newp)
            if mp is not p:
                p.copy_(newp)


def fused_momentum_(params, grads, velocities, masters, lr, mu, use_nesterov=False, weight_decay=0.0,
                    lr_ratios=None, grad_scale=1.0):
    if params and _use_hip(params[0]):
        return _hip.multi_tensor_momentum(params, grads, velocities, masters, lr, mu, use_nesterov,
                                          weight_decay, lr_ratios, grad_scale)
    with torch.no_grad():
        for i, (p, g, vel) in enumerate(zip(params, grads, velocities)):
            if g is None:
                continue
            mp = masters[i] if masters is not None and masters[i] is not None else p
            lr_i = lr * (lr_ratios[i] if lr_ratios is not None else 1.0)
            gf = g.float() * grad_scale
            if weight_decay:
                gf = gf + weight_decay * mp.float()
            vel.mul_(mu).add_(gf)
            if use_nesterov:
                newp = mp.float() - lr_i * (gf + mu * vel)
            else:
                newp = mp.float() - lr_i * vel
            mp.copy_(newp)
            if mp is not p:
                p.copy_(newp)


def global_norm_sq(tensors):
    """Sum of squares over a list of tensors (fp32 scalar tensor)."""
    tensors = [t for t in tensors if t is not None]
    if not tensors:
        return torch.zeros((), dtype=torch.float32)
    if _use_hip(tensors[0]):
        return _hip.multi_tensor_l2norm_sq(tensors)
    return sum(t.float().pow(2).sum() for t in tensors)


def scale_grads_(tensors, scale):
    with torch.no_grad():
        torch._foreach_mul_([t for t in tensors if t is not None], scale)


def check_finite_and_unscale_(tensors, inv_scale):
    """Unscale in place; return a bool tensor ``found_inf`` (reference: operators/amp/check_finite_and_unscale_op.cu)."""
    tensors = [t for t in tensors if t is not None]
    if not tensors:
        return torch.zeros((), dtype=torch.bool)
    found = torch.zeros(1, dtype=torch.float32, device=tensors[0].device)
    torch._amp_foreach_non_finite_check_and_unscale_(tensors, found, torch.tensor([inv_scale], dtype=torch.float32, device=tensors[0].device))
    return found[0] > 0


# ----------------------------------------------------------------------------
# batch norm (training stats) — NHWC channel reduction
# ----------------------------------------------------------------------------
class _BatchNormNHWC(torch.autograd.Function):
    """Training batch norm over the last (channel) dim with optional fused residual add + ReLU
    (HIP kernels in csrc/kernels/batch_norm.hip)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, momentum, eps, relu):
        w32 = weight.float() if weight is not None else torch.ones(x.shape[-1], device=x.device)
        b32 = bias.float() if bias is not None else None
        ext = getattr(x, "_pha_bn_stats", None)   # partial sums from the producing conv's epilogue
        if ext is not None and (ext[2] != x._version or ext[0].device != x.device or ext[1] <= 0):
            ext = None
        y, mean, istd, aff = _hip.bn_fwd_train(x, w32, b32, running_mean, running_var, eps, momentum, residual,
                                               relu, ext_stats=None if ext is None else (ext[0], ext[1]))
        # ReLU without a residual: the backward recomputes the mask from x and the affine, y is not kept
        keep_y = relu and residual is not None
        ctx.save_for_backward(x, y if keep_y else None, w32, mean, istd, aff if relu else None)
        if residual is None:
            # the convolution consuming y can reduce this BN's backward sums in its dgrad epilogue
            ctx.bn_token = object()
            y._pha_bn_src = (x, mean, aff if relu else None, ctx.bn_token)
        ctx.relu, ctx.has_res = relu, residual is not None
        # residual-gradient route (conv_gemm.res_route_begin): the residual is a block input whose
        # other consumer, an armed conv, adds this gradient in its dgrad epilogue
        route = getattr(residual, "_pha_res_route", None) if residual is not None else None
        ctx.route = None
        if route is not None and route.get("armed") and not route.get("sink"):
            route["sink"] = True
            ctx.route = route
        ctx.wdt = None if weight is None else weight.dtype
        ctx.bdt = None if bias is None else bias.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, w32, mean, istd, aff = ctx.saved_tensors
        ext = getattr(gy, "_pha_bn_bwd", None)   # sums from the producing dgrad's epilogue
        if ext is not None and (ext[2] is not getattr(ctx, "bn_token", None) or ext[3] != gy._version):
            ext = None
        dx, dw, db, dres = _hip.bn_bwd(gy.contiguous(), x, y, w32, mean, istd, ctx.relu, ctx.has_res, affine=aff,
                                       ext_part=None if ext is None else (ext[0], ext[1]))
        if ctx.route is not None and dres is not None:
            ctx.route["g"] = dres   # handed to the armed conv's dgrad epilogue
            dres = None
        return (dx, None if ctx.wdt is None else dw.to(ctx.wdt), None if ctx.bdt is None else db.to(ctx.bdt),
                None, None, dres, None, None, None)


def _bn_hip_ok(x, channel_axis):
    return (_use_hip(x) and channel_axis in (-1, x.dim() - 1) and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.is_contiguous() and x.shape[-1] % 8 == 0 and x.numel() > 0)


def batch_norm_train(x, weight, bias, running_mean, running_var, momentum, eps, channel_axis, residual=None,
                     relu=False):
    """Training-mode BN (Paddle momentum semantics: running = running*m + batch*(1-m)).
    Channels-last inputs use the fused HIP kernels; other layouts fall back to torch."""
    if _bn_hip_ok(x, channel_axis) and (running_mean is None or running_mean.dtype == torch.float32) and \
            (residual is None or (residual.dtype == x.dtype and residual.shape == x.shape)):
        res = residual.contiguous() if residual is not None else None
        return _BatchNormNHWC.apply(x, weight, bias, running_mean, running_var, res, float(momentum), float(eps),
                                    bool(relu))
    if channel_axis in (-1, x.dim() - 1) and x.dim() > 2:
        perm = [0, x.dim() - 1] + list(range(1, x.dim() - 1))
        xt = x.permute(*perm)
        y = TF.batch_norm(xt, running_mean, running_var, weight, bias, True, 1 - momentum, eps)
        inv = [0] + list(range(2, x.dim())) + [1]
        y = y.permute(*inv)
    else:
        y = TF.batch_norm(x, running_mean, running_var, weight, bias, True, 1 - momentum, eps)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y


def batch_norm_infer(x, weight, bias, running_mean, running_var, eps, channel_axis, residual=None, relu=False):
    """Eval-mode BN (frozen statistics) as one fused affine (+add)(+relu) pass."""
    if _bn_hip_ok(x, channel_axis) and (residual is None or (residual.dtype == x.dtype and residual.shape == x.shape)):
        istd = torch.rsqrt(running_var.float() + eps)
        scale = istd * (weight.float() if weight is not None else 1.0)
        shift = (bias.float() if bias is not None else 0.0) - running_mean.float() * scale
        if not torch.is_grad_enabled() or not (x.requires_grad or (weight is not None and weight.requires_grad)):
            return _hip.bn_apply(x, scale.contiguous(), shift.contiguous(),
                                 residual.contiguous() if residual is not None else None, relu)
    shape = [1] * (x.dim() - 1) + [-1] if channel_axis in (-1, x.dim() - 1) else [1, -1] + [1] * (x.dim() - 2)
    istd = torch.rsqrt(running_var + eps)
    y = (x - running_mean.reshape(shape)) * istd.reshape(shape)
    if weight is not None:
        y = y * weight.reshape(shape)
    if bias is not None:
        y = y + bias.reshape(shape)
    y = y.to(x.dtype)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y
