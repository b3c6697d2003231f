"""Fused transformer functionals (reference: python/paddle/incubate/nn/functional/
fused_transformer.py, fused_matmul_bias.py).

The reference fuses these into single CUDA ops; here each maps onto the MI355X kernel set:
GEMMs on hipBLASLt (with the bias folded into the GEMM via ``addmm``), attention on the
MFMA flash-attention HIP kernel when there is no arbitrary additive mask (masked attention
falls back to fused SDPA), LayerNorm / bias-GELU on the HIP kernels. Weight layouts and
return values follow the reference exactly (qkv_weight [3, H, D, E]; cache_kv
[2, B, H, S, D])."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _wrap
from ... import ops as _ops

__all__ = ["fused_multi_head_attention", "fused_feedforward", "fused_multi_transformer", "fused_matmul_bias",
           "fused_linear", "fused_bias_dropout_residual_layer_norm"]


def _u(x):
    return None if x is None else (x._t if isinstance(x, Tensor) else x)


def _dropout(x, p, training, mode):
    if p == 0.0:
        return x
    if training:
        if mode in ("upscale_in_train", "upscale-in-train"):
            return TF.dropout(x, p, True)
        return x * (torch.rand_like(x) >= p).to(x.dtype)
    return x if mode in ("upscale_in_train", "upscale-in-train") else x * (1.0 - p)


def _ln(x, w, b, eps):
    if w is None and b is None:
        return TF.layer_norm(x, [x.shape[-1]], None, None, eps)
    w = w if w is not None else torch.ones(x.shape[-1], dtype=x.dtype, device=x.device)
    return _ops.fused.layer_norm(x, [x.shape[-1]], w.to(x.dtype) if w.dtype != x.dtype and w.dtype != torch.float32 else w,
                                 None if b is None else b.to(w.dtype), eps)


def _act(x, bias, activation):
    if activation == "gelu":
        return _ops.fused.bias_gelu(x, bias, False) if bias is not None else _ops.fused.gelu(x, False)
    h = x + bias if bias is not None else x
    if activation == "relu":
        return torch.relu(h)
    raise ValueError(f"unsupported activation {activation}")


def fused_matmul_bias(x, y, bias=None, transpose_x=False, transpose_y=False, name=None):
    a, b = _u(x), _u(y)
    if transpose_x:
        a = a.transpose(-1, -2)
    if transpose_y:
        b = b.transpose(-1, -2)
    if bias is not None and a.dim() == 2:
        return _wrap(torch.addmm(_u(bias), a, b))
    out = torch.matmul(a, b)
    return _wrap(out + _u(bias) if bias is not None else out)


def fused_linear(x, weight, bias=None, transpose_weight=False, name=None):
    return fused_matmul_bias(x, weight, bias, False, transpose_weight)


def _linear(x, w, b):
    if b is not None:
        return torch.addmm(b, x.reshape(-1, x.shape[-1]), w).reshape(*x.shape[:-1], w.shape[-1])
    return x @ w


def fused_bias_dropout_residual_layer_norm(x, residual, bias=None, ln_scale=None, ln_bias=None, dropout_rate=0.5,
                                           ln_epsilon=1e-5, training=True, mode="upscale_in_train", name=None):
    h = _u(x)
    if mode in ("upscale_in_train", "upscale-in-train") or not training or dropout_rate == 0.0:
        # one fused HIP pass each way (ops/fused.py _BiasDropoutResidualLN); eval-mode upscale dropout is identity
        w = _u(ln_scale)
        w = w if w is not None else torch.ones(h.shape[-1], dtype=torch.float32, device=h.device)
        r = _u(residual)
        return _wrap(_ops.fused.bias_dropout_residual_layer_norm(h.contiguous(), r.contiguous().to(h.dtype), _u(bias), w,
                                                                 _u(ln_bias), dropout_rate, training, ln_epsilon))
    if bias is not None:
        h = h + _u(bias)
    h = _dropout(h, dropout_rate, training, mode) + _u(residual)
    return _wrap(_ln(h, _u(ln_scale), _u(ln_bias), ln_epsilon))


def fused_feedforward(x, linear1_weight, linear2_weight, linear1_bias=None, linear2_bias=None, ln1_scale=None,
                      ln1_bias=None, ln2_scale=None, ln2_bias=None, dropout1_rate=0.5, dropout2_rate=0.5,
                      activation="relu", ln1_epsilon=1e-5, ln2_epsilon=1e-5, pre_layer_norm=False, training=True,
                      mode="upscale_in_train", ring_id=-1, add_residual=True, name=None):
    t = _u(x)
    residual = t
    h = _ln(t, _u(ln1_scale), _u(ln1_bias), ln1_epsilon) if pre_layer_norm else t
    h = _act(h @ _u(linear1_weight), _u(linear1_bias), activation)
    h = _dropout(h, dropout1_rate, training, mode)
    h = _linear(h, _u(linear2_weight), _u(linear2_bias))
    if ring_id >= 0:
        from ...parallel import collective as C
        torch.distributed.all_reduce(h)
    if (not pre_layer_norm and add_residual and
            (mode in ("upscale_in_train", "upscale-in-train") or not training or dropout2_rate == 0.0)):
        w = _u(ln2_scale)
        w = w if w is not None else torch.ones(h.shape[-1], dtype=torch.float32, device=h.device)
        return _wrap(_ops.fused.bias_dropout_residual_layer_norm(h.contiguous(), residual.contiguous(), None, w,
                                                                 _u(ln2_bias), dropout2_rate, training, ln2_epsilon))
    h = _dropout(h, dropout2_rate, training, mode)
    if add_residual:
        h = residual + h
    if not pre_layer_norm:
        h = _ln(h, _u(ln2_scale), _u(ln2_bias), ln2_epsilon)
    return _wrap(h)


def _attention(q, k, v, mask, attn_dropout, training, mode, causal=False):
    """q/k/v: [B, H, S, D]. The flash kernels (mask and upscale-in-train dropout in-kernel); the
    downscale-in-infer dropout mode keeps the explicit composite."""
    if mode in ("upscale_in_train", "upscale-in-train") or attn_dropout == 0.0 or not training:
        o = _ops.fused.flash_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), causal=causal,
                                       dropout_p=attn_dropout, training=training, mask=mask)
        return o.transpose(1, 2)
    if mode not in ("upscale_in_train", "upscale-in-train") and attn_dropout > 0:
        s = (q @ k.transpose(-1, -2)) / (q.shape[-1] ** 0.5)
        if mask is not None:
            s = s + mask
        p = _dropout(torch.softmax(s.float(), -1).to(q.dtype), attn_dropout, training, mode)
        return p @ v
    return TF.scaled_dot_product_attention(q, k, v, attn_mask=mask.to(q.dtype) if mask is not None else None,
                                           dropout_p=attn_dropout if training else 0.0, is_causal=causal and mask is None)


def fused_multi_head_attention(x, qkv_weight, linear_weight, pre_layer_norm=False, pre_ln_scale=None,
                               pre_ln_bias=None, ln_scale=None, ln_bias=None, pre_ln_epsilon=1e-05, qkv_bias=None,
                               linear_bias=None, cache_kv=None, attn_mask=None, dropout_rate=0.5,
                               attn_dropout_rate=0.5, ln_epsilon=1e-05, training=True, mode="upscale_in_train",
                               ring_id=-1, add_residual=True, name=None):
    t = _u(x)
    B, S, E = t.shape
    w = _u(qkv_weight)  # [3, H, D, E]
    _, H, D, _ = w.shape
    residual = t
    h = _ln(t, _u(pre_ln_scale), _u(pre_ln_bias), pre_ln_epsilon) if pre_layer_norm else t
    qkv = h.reshape(B * S, E) @ w.reshape(3 * H * D, E).t()
    if qkv_bias is not None:
        qkv = qkv + _u(qkv_bias).reshape(-1)
    qkv = qkv.reshape(B, S, 3, H, D).permute(2, 0, 3, 1, 4)  # [3, B, H, S, D]
    q, k, v = qkv[0], qkv[1], qkv[2]
    cache_out = None
    if cache_kv is not None:
        c = _u(cache_kv)
        k = torch.cat([c[0], k], 2)
        v = torch.cat([c[1], v], 2)
        cache_out = torch.stack([k, v], 0)
    o = _attention(q, k, v, _u(attn_mask), attn_dropout_rate, training, mode)
    o = o.transpose(1, 2).reshape(B, S, H * D)
    o = _linear(o, _u(linear_weight), _u(linear_bias))
    if ring_id >= 0:
        torch.distributed.all_reduce(o)
    o = _dropout(o, dropout_rate, training, mode)
    if add_residual:
        o = residual + o
    if not pre_layer_norm:
        o = _ln(o, _u(ln_scale), _u(ln_bias), ln_epsilon)
    if cache_kv is not None:
        return _wrap(o), _wrap(cache_out)
    return _wrap(o)


def fused_multi_transformer(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights, linear_biases,
                            ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases, ffn2_weights, ffn2_biases,
                            pre_layer_norm=True, epsilon=1e-05, cache_kvs=None, time_step=None, attn_mask=None,
                            dropout_rate=0.0, activation="gelu", training=False, mode="upscale_in_train",
                            trans_qkvw=True, ring_id=-1, name=None):
    """Stack of pre-LN decoder layers for generation. ``cache_kvs[i]`` is a preallocated
    [2, B, H, max_seq, D] buffer updated in place: context stage (time_step None) writes
    positions [0, S); decode stage (S == 1) writes position ``time_step`` and attends over
    [0, time_step]."""
    h = _u(x)
    B, S, E = h.shape
    ts = None
    if time_step is not None:
        ts = int(_u(time_step).reshape(-1)[0].item()) if isinstance(time_step, (Tensor, torch.Tensor)) else int(time_step)
    mask = _u(attn_mask)
    for i in range(len(qkv_weights)):
        residual = h
        a = _ln(h, _u(ln_scales[i]), _u(ln_biases[i]), epsilon) if pre_layer_norm else h
        w = _u(qkv_weights[i])
        if trans_qkvw:  # [3, H, D, E]
            _, H, D, _ = w.shape
            qkv = a.reshape(B * S, E) @ w.reshape(3 * H * D, E).t()
        else:  # [E, 3, H, D]
            _, _, H, D = w.shape
            qkv = a.reshape(B * S, E) @ w.reshape(E, 3 * H * D)
        if qkv_biases is not None and qkv_biases[i] is not None:
            qkv = qkv + _u(qkv_biases[i]).reshape(-1)
        qkv = qkv.reshape(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        causal = False
        if cache_kvs is not None:
            c = _u(cache_kvs[i])
            if ts is None:
                c[0, :, :, :S] = k
                c[1, :, :, :S] = v
                causal = mask is None
            else:
                c[0, :, :, ts:ts + S] = k
                c[1, :, :, ts:ts + S] = v
                k, v = c[0, :, :, :ts + S], c[1, :, :, :ts + S]
        m = mask
        if m is not None and m.shape[-1] != k.shape[2]:
            m = m[..., :k.shape[2]]
        o = _attention(q, k, v, m, dropout_rate, training, mode, causal=causal and S > 1)
        o = o.transpose(1, 2).reshape(B, S, H * D)
        o = _linear(o, _u(linear_weights[i]), _u(linear_biases[i]) if linear_biases is not None else None)
        if ring_id >= 0:
            torch.distributed.all_reduce(o)
        h = residual + _dropout(o, dropout_rate, training, mode)
        if not pre_layer_norm:
            h = _ln(h, _u(ln_scales[i]), _u(ln_biases[i]), epsilon)
        residual = h
        f = _ln(h, _u(ffn_ln_scales[i]), _u(ffn_ln_biases[i]), epsilon) if pre_layer_norm else h
        f = _act(f @ _u(ffn1_weights[i]), _u(ffn1_biases[i]) if ffn1_biases is not None else None, activation)
        f = _linear(f, _u(ffn2_weights[i]), _u(ffn2_biases[i]) if ffn2_biases is not None else None)
        if ring_id >= 0:
            torch.distributed.all_reduce(f)
        h = residual + _dropout(f, dropout_rate, training, mode)
        if not pre_layer_norm:
            h = _ln(h, _u(ffn_ln_scales[i]), _u(ffn_ln_biases[i]), epsilon)
    if cache_kvs is not None:
        return _wrap(h), cache_kvs
    return _wrap(h)
