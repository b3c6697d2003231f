"""Transformer layers (reference: python/paddle/nn/layer/transformer.py).

Structure and parameter names match the reference (``q_proj``/``k_proj``/
``v_proj``/``out_proj``, ``linear1``/``linear2``, ``norm1``/``norm2``…).
Attention without an explicit mask and without returned weights runs the
MFMA flash-attention kernel; masked attention takes the SDPA path.
"""
from __future__ import annotations

import collections
import copy

import torch

from ...framework.core import Tensor, _wrap
from ...framework.param_attr import ParamAttr
from .. import functional as F
from .common import Linear, Dropout
from .conv_norm_pool import LayerNorm
from .container import LayerList
from .layers import Layer

__all__ = ["MultiHeadAttention", "TransformerEncoderLayer", "TransformerEncoder", "TransformerDecoderLayer",
           "TransformerDecoder", "Transformer"]


def _convert_attn_mask(mask, dtype):
    if mask is None:
        return None
    m = mask._t
    if m.dtype == torch.bool or m.dtype in (torch.int32, torch.int64, torch.uint8):
        return m.to(torch.bool)
    return m.to(dtype)


def _attr_list(attr, n):
    if isinstance(attr, (list, tuple)):
        assert len(attr) == n
        return list(attr)
    return [attr] * n


class MultiHeadAttention(Layer):
    Cache = collections.namedtuple("Cache", ["k", "v"])
    StaticCache = collections.namedtuple("StaticCache", ["k", "v"])

    def __init__(self, embed_dim, num_heads, dropout=0.0, kdim=None, vdim=None, need_weights=False,
                 weight_attr=None, bias_attr=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.kdim, self.vdim = kdim or embed_dim, vdim or embed_dim
        self.dropout, self.need_weights = dropout, need_weights
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == embed_dim
        self.q_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr=bias_attr)
        self.k_proj = Linear(self.kdim, embed_dim, weight_attr, bias_attr=bias_attr)
        self.v_proj = Linear(self.vdim, embed_dim, weight_attr, bias_attr=bias_attr)
        self.out_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr=bias_attr)

    def _split(self, t):
        B, S, _ = t.shape
        return t.reshape(B, S, self.num_heads, self.head_dim)

    def compute_kv(self, key, value):
        k = self._split(self.k_proj(key)._t)
        v = self._split(self.v_proj(value)._t)
        return k, v

    def gen_cache(self, key, value=None, type=Cache):
        if type == MultiHeadAttention.StaticCache:
            k, v = self.compute_kv(key, value if value is not None else key)
            return self.StaticCache(_wrap(k), _wrap(v))
        if value is None:
            B = key._t.shape[0]
            z = torch.zeros(B, 0, self.num_heads, self.head_dim, dtype=key._t.dtype, device=key._t.device)
            return self.Cache(_wrap(z), _wrap(z.clone()))
        return self.Cache(key, value)

    def _forward_ops(self, query, key, value, attn_mask, cache):
        """the reference's op-level graph (nn/layer/transformer.py MultiHeadAttention.forward:
        projections, reshape2 / transpose2 to [B, H, S, D], scaled matmul_v2, mask add, softmax,
        dropout, matmul_v2, transpose2 / reshape2, out projection): what static Programs
        (jit.save, to_static) record, so a saved model holds reference op types"""
        from ... import tensor as T

        def heads(t):
            return T.transpose(T.reshape(t, [0, 0, self.num_heads, self.head_dim]), [0, 2, 1, 3])
        q = heads(self.q_proj(query))
        if isinstance(cache, self.StaticCache):
            k, v = cache.k, cache.v
        else:
            k, v = heads(self.k_proj(key)), heads(self.v_proj(value))
        if isinstance(cache, self.Cache):
            k, v = T.concat([cache.k, k], axis=2), T.concat([cache.v, v], axis=2)
            cache = self.Cache(k, v)
        product = T.matmul(T.scale(q, self.head_dim ** -0.5), k, transpose_y=True)
        if attn_mask is not None:
            m = attn_mask
            if str(m.dtype).endswith(("bool", "int32", "int64", "uint8")):
                m = T.scale(T.cast(m, product.dtype), 1e9, bias=-1e9)   # keep 0, masked -1e9
            product = product + m
        weights = F.softmax(product)
        if self.dropout:
            weights = F.dropout(weights, self.dropout, training=self.training, mode="upscale_in_train")
        out = T.reshape(T.transpose(T.matmul(weights, v), [0, 2, 1, 3]), [0, 0, self.embed_dim])
        outs = [self.out_proj(out)]
        if self.need_weights:
            outs.append(weights)
        if cache is not None:
            outs.append(cache)
        return outs[0] if len(outs) == 1 else tuple(outs)

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        key = query if key is None else key
        value = query if value is None else value
        from ...framework.core import _mode
        if _mode.static:
            return self._forward_ops(query, key, value, attn_mask, cache)
        q = self._split(self.q_proj(query)._t)
        if isinstance(cache, self.StaticCache):
            k, v = cache.k._t, cache.v._t
        else:
            k, v = self.compute_kv(key, value)
        if isinstance(cache, self.Cache):
            k = torch.cat([cache.k._t, k], 1)
            v = torch.cat([cache.v._t, v], 1)
            cache = self.Cache(_wrap(k), _wrap(v))
        mask = _convert_attn_mask(attn_mask, q.dtype)
        drop = self.dropout if self.training else 0.0
        weights = None
        if not self.need_weights:
            # mask and attention dropout run inside the flash kernels (the probabilities are
            # never materialised); only need_weights=True keeps the explicit composite
            from ... import ops
            out = ops.flash_attention(q, k, v, False, drop, None, self.training, mask=mask)
        else:
            qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
            scores = torch.matmul(qt, kt.transpose(-1, -2)) * (self.head_dim ** -0.5)
            if mask is not None:
                if mask.dtype == torch.bool:
                    scores = scores.masked_fill(~mask, float("-inf"))
                else:
                    scores = scores + mask
            p = torch.softmax(scores.float(), -1).to(q.dtype)
            if drop:
                p = torch.nn.functional.dropout(p, drop, True)
            weights = p
            out = torch.matmul(p, vt).transpose(1, 2)
        B, S = out.shape[:2]
        out = self.out_proj(_wrap(out.reshape(B, S, self.embed_dim)))
        outs = [out]
        if self.need_weights:
            outs.append(_wrap(weights))
        if cache is not None:
            outs.append(cache)
        return out if len(outs) == 1 else tuple(outs)


class TransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        w = _attr_list(weight_attr, 2)
        b = _attr_list(bias_attr, 2)
        self.self_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=w[0], bias_attr=b[0])
        self.linear1 = Linear(d_model, dim_feedforward, w[1], bias_attr=b[1])
        self.dropout = Dropout(act_dropout, mode="upscale_in_train")
        self.linear2 = Linear(dim_feedforward, d_model, w[1], bias_attr=b[1])
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout, mode="upscale_in_train")
        self.dropout2 = Dropout(dropout, mode="upscale_in_train")
        self.activation = activation

    def _ffn_act(self, x):
        from ...framework.core import _mode
        if self.activation == "gelu" and not _mode.static:
            from ... import ops
            h = torch.matmul(x._t, self.linear1.weight._t)
            return _wrap(ops.bias_gelu(h, self.linear1.bias._t)) if self.linear1.bias is not None else F.gelu(_wrap(h))
        return getattr(F, self.activation)(self.linear1(x))

    def forward(self, src, src_mask=None, cache=None):
        residual = src
        if self.normalize_before:
            src = self.norm1(src)
        if cache is None:
            src = self.self_attn(src, src, src, src_mask)
        else:
            src, incremental_cache = self.self_attn(src, src, src, src_mask, cache)
        src = residual + self.dropout1(src)
        if not self.normalize_before:
            src = self.norm1(src)
        residual = src
        if self.normalize_before:
            src = self.norm2(src)
        src = self.linear2(self.dropout(self._ffn_act(src)))
        src = residual + self.dropout2(src)
        if not self.normalize_before:
            src = self.norm2(src)
        return src if cache is None else (src, incremental_cache)

    def gen_cache(self, src):
        return self.self_attn.gen_cache(src, type=self.self_attn.Cache)


class TransformerEncoder(Layer):
    def __init__(self, encoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([encoder_layer if i == 0 else copy.deepcopy(encoder_layer) for i in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm

    def forward(self, src, src_mask=None, cache=None):
        output = src
        new_caches = []
        for i, mod in enumerate(self.layers):
            if cache is None:
                output = mod(output, src_mask=src_mask)
            else:
                output, c = mod(output, src_mask=src_mask, cache=cache[i])
                new_caches.append(c)
        if self.norm is not None:
            output = self.norm(output)
        return output if cache is None else (output, new_caches)

    def gen_cache(self, src):
        return [layer.gen_cache(src) for layer in self.layers]


class TransformerDecoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        w = _attr_list(weight_attr, 3)
        b = _attr_list(bias_attr, 3)
        self.self_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=w[0], bias_attr=b[0])
        self.cross_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=w[1], bias_attr=b[1])
        self.linear1 = Linear(d_model, dim_feedforward, w[2], bias_attr=b[2])
        self.dropout = Dropout(act_dropout, mode="upscale_in_train")
        self.linear2 = Linear(dim_feedforward, d_model, w[2], bias_attr=b[2])
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.norm3 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout, mode="upscale_in_train")
        self.dropout2 = Dropout(dropout, mode="upscale_in_train")
        self.dropout3 = Dropout(dropout, mode="upscale_in_train")
        self.activation = activation

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        residual = tgt
        if self.normalize_before:
            tgt = self.norm1(tgt)
        if cache is None:
            tgt = self.self_attn(tgt, tgt, tgt, tgt_mask, None)
        else:
            tgt, incremental_cache = self.self_attn(tgt, tgt, tgt, tgt_mask, cache[0])
        tgt = residual + self.dropout1(tgt)
        if not self.normalize_before:
            tgt = self.norm1(tgt)
        residual = tgt
        if self.normalize_before:
            tgt = self.norm2(tgt)
        if cache is None:
            tgt = self.cross_attn(tgt, memory, memory, memory_mask, None)
        else:
            tgt, static_cache = self.cross_attn(tgt, memory, memory, memory_mask, cache[1])
        tgt = residual + self.dropout2(tgt)
        if not self.normalize_before:
            tgt = self.norm2(tgt)
        residual = tgt
        if self.normalize_before:
            tgt = self.norm3(tgt)
        tgt = self.linear2(self.dropout(getattr(F, self.activation)(self.linear1(tgt))))
        tgt = residual + self.dropout3(tgt)
        if not self.normalize_before:
            tgt = self.norm3(tgt)
        return tgt if cache is None else (tgt, (incremental_cache, static_cache))

    def gen_cache(self, memory):
        inc = self.self_attn.gen_cache(memory, type=self.self_attn.Cache)
        static = self.cross_attn.gen_cache(memory, memory, type=self.cross_attn.StaticCache)
        return inc, static


class TransformerDecoder(Layer):
    def __init__(self, decoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([decoder_layer if i == 0 else copy.deepcopy(decoder_layer) for i in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        output = tgt
        new_caches = []
        for i, mod in enumerate(self.layers):
            if cache is None:
                output = mod(output, memory, tgt_mask=tgt_mask, memory_mask=memory_mask, cache=None)
            else:
                output, c = mod(output, memory, tgt_mask=tgt_mask, memory_mask=memory_mask, cache=cache[i])
                new_caches.append(c)
        if self.norm is not None:
            output = self.norm(output)
        return output if cache is None else (output, new_caches)

    def gen_cache(self, memory, do_zip=False):
        cache = [layer.gen_cache(memory) for layer in self.layers]
        if do_zip:
            cache = list(zip(*cache))
        return cache


class Transformer(Layer):
    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=2048,
                 dropout=0.1, activation="relu", attn_dropout=None, act_dropout=None, normalize_before=False,
                 weight_attr=None, bias_attr=None, custom_encoder=None, custom_decoder=None):
        super().__init__()
        if custom_encoder is not None:
            self.encoder = custom_encoder
        else:
            enc = TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout, act_dropout,
                                          normalize_before, weight_attr, bias_attr)
            self.encoder = TransformerEncoder(enc, num_encoder_layers, LayerNorm(d_model) if normalize_before else None)
        if custom_decoder is not None:
            self.decoder = custom_decoder
        else:
            dec = TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout, act_dropout,
                                          normalize_before, weight_attr, bias_attr)
            self.decoder = TransformerDecoder(dec, num_decoder_layers, LayerNorm(d_model) if normalize_before else None)
        self.d_model, self.nhead = d_model, nhead

    def forward(self, src, tgt, src_mask=None, tgt_mask=None, memory_mask=None):
        memory = self.encoder(src, src_mask=src_mask)
        return self.decoder(tgt, memory, tgt_mask=tgt_mask, memory_mask=memory_mask)

    @staticmethod
    def generate_square_subsequent_mask(length):
        from ...framework import core
        m = torch.triu(torch.full((length, length), float("-inf"), device=core.default_device()), 1)
        return _wrap(m)
