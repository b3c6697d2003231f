"""Attention functionals (reference: python/paddle/nn/functional/sparse_attention.py,
python/paddle/incubate/nn/functional/fused_transformer.py, operators/fused/fmha_ref.h).

``scaled_dot_product_attention`` / ``flash_attention`` take Paddle's
[batch, seq, heads, head_dim] layout and run our MFMA flash-attention kernel on
gfx950 (ops.flash_attention)."""
from __future__ import annotations

import math

import torch

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops
from ... import ops as _ops

_w = _wrap

__all__ = ["scaled_dot_product_attention", "flash_attention", "sparse_attention"]


def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False,
                                 training=True, name=None, scale=None):
    q, k, v = query._t, key._t, value._t
    m = None if attn_mask is None else attn_mask._t
    return _w(_ops.flash_attention(q, k, v, is_causal, dropout_p, scale, training, mask=m))


def flash_attention(query, key, value, dropout=0.0, causal=False, return_softmax=False, fixed_seed_offset=None,
                    rng_name="", training=True, name=None):
    out = _w(_ops.flash_attention(query._t, key._t, value._t, causal, dropout, None, training))
    return out, None


def sparse_attention(query, key, value, sparse_csr_offset, sparse_csr_columns, key_padding_mask=None,
                     attn_mask=None, name=None):
    """CSR block-sparse attention: q,k,v [B, H, S, D]; offsets [B, H, S+1]; columns [B, H, nnz]."""
    q, k, v = query._t, key._t, value._t
    B, H, S, D = q.shape
    off = sparse_csr_offset._t.long()
    cols = sparse_csr_columns._t.long()
    dense = torch.zeros(B, H, S, S, dtype=torch.bool, device=q.device)
    for b in range(B):
        for h in range(H):
            o = off[b, h]
            rows = torch.repeat_interleave(torch.arange(S, device=q.device), o[1:] - o[:-1])
            dense[b, h, rows, cols[b, h, : rows.numel()]] = True
    scores = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(D)
    scores = scores.masked_fill(~dense, float("-inf"))
    if key_padding_mask is not None:
        scores = scores + key_padding_mask._t.reshape(B, 1, 1, S)
    if attn_mask is not None:
        scores = scores + attn_mask._t.reshape(1, 1, S, S)
    p = torch.softmax(scores.float(), -1).to(q.dtype)
    p = torch.nan_to_num(p)
    return _w(torch.matmul(p, v))


register_ops(globals(), __all__)
