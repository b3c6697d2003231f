"""GPT (GPT-3 family) for fleet training — the model behind the headline
"tokens/sec GPT-3 1.3B" benchmark (reference usage: the fleet hybrid-parallel GPT
tests, python/paddle/fluid/tests/unittests/hybrid_parallel_pp_transformer.py,
and PaddleNLP/fleetx GPT whose parameter layout this follows).

MI355X-first choices:
  * pre-LN decoder; fused QKV projection (one [h, 3h] GEMM on hipBLASLt);
  * attention = our MFMA flash-attention kernel on [B, S, H, D] (no S×S tensor);
  * FFN = GEMM + fused bias-GELU HIP kernel + GEMM;
  * LayerNorm = HIP wave-per-row kernel; loss = fused one-pass softmax-CE kernel
    over the (tied-embedding) vocab logits;
  * tensor parallel: QKV/FFN1 column-parallel, out/FFN2 row-parallel, vocab-parallel
    embedding + parallel cross-entropy when ``tensor_parallel_degree > 1``;
  * optional activation recompute per layer (``recompute=True``).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from ..framework.core import Tensor, _wrap
from .. import nn
from ..nn import functional as F
from ..nn import initializer as I
from .. import ops as _ops
from ..ops import conv_gemm as _cg


@dataclass
class GPTConfig:
    vocab_size: int = 50304
    hidden_size: int = 2048
    num_layers: int = 24
    num_heads: int = 16
    ffn_hidden_size: int = 8192
    max_position_embeddings: int = 2048
    hidden_dropout: float = 0.0
    attention_dropout: float = 0.0
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-5
    tensor_parallel_degree: int = 1
    recompute: bool = False
    fuse_qkv: bool = True
    tie_word_embeddings: bool = True

    @property
    def head_dim(self):
        return self.hidden_size // self.num_heads


GPT_CONFIGS = {
    "gpt3-125m": dict(hidden_size=768, num_layers=12, num_heads=12, ffn_hidden_size=3072),
    "gpt3-350m": dict(hidden_size=1024, num_layers=24, num_heads=16, ffn_hidden_size=4096),
    "gpt3-1.3b": dict(hidden_size=2048, num_layers=24, num_heads=16, ffn_hidden_size=8192),
    "gpt3-2.7b": dict(hidden_size=2560, num_layers=32, num_heads=32, ffn_hidden_size=10240),
    "gpt3-6.7b": dict(hidden_size=4096, num_layers=32, num_heads=32, ffn_hidden_size=16384),
    "gpt3-13b": dict(hidden_size=5120, num_layers=40, num_heads=40, ffn_hidden_size=20480),
    "gpt-tiny": dict(hidden_size=64, num_layers=2, num_heads=4, ffn_hidden_size=256, vocab_size=512,
                     max_position_embeddings=128),
}


def gpt_config(name, **overrides):
    d = dict(GPT_CONFIGS[name])
    d.update(overrides)
    return GPTConfig(**d)


def _w_attr(cfg, scale=1.0):
    return nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range * scale))


class GPTAttention(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.cfg = cfg
        h = cfg.hidden_size
        tp = cfg.tensor_parallel_degree
        self.num_heads = cfg.num_heads // tp
        self.head_dim = cfg.head_dim
        out_scale = 1.0 / math.sqrt(2.0 * cfg.num_layers)
        if tp > 1:
            from ..parallel.mp_layers import ColumnParallelLinear, RowParallelLinear
            self.qkv_proj = ColumnParallelLinear(h, 3 * h, weight_attr=_w_attr(cfg), has_bias=True, gather_output=False)
            self.out_proj = RowParallelLinear(h, h, weight_attr=_w_attr(cfg, out_scale), has_bias=True, input_is_parallel=True)
        else:
            self.qkv_proj = nn.Linear(h, 3 * h, weight_attr=_w_attr(cfg))
            self.out_proj = nn.Linear(h, h, weight_attr=_w_attr(cfg, out_scale))

    def forward(self, x, defer_bias=False):
        """defer_bias: return (projection without its bias, the bias) for the next add-LN kernel
        to add (its backward then yields the bias gradient as a by-product)"""
        B, S = x._t.shape[0], x._t.shape[1]
        qkv = self.qkv_proj(x)._t.reshape(B, S, self.num_heads, 3 * self.head_dim)
        drop = self.cfg.attention_dropout if self.training else 0.0
        o = _ops.fused.flash_attention_qkvpacked(qkv, self.num_heads, causal=True, dropout_p=drop,
                                                 training=self.training)
        o = _wrap(o.reshape(B, S, self.num_heads * self.head_dim))
        if defer_bias and self.cfg.tensor_parallel_degree <= 1:
            return F.linear(o, self.out_proj.weight, None), self.out_proj.bias
        return self.out_proj(o)


class GPTMLP(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.cfg = cfg
        h, f = cfg.hidden_size, cfg.ffn_hidden_size
        out_scale = 1.0 / math.sqrt(2.0 * cfg.num_layers)
        if cfg.tensor_parallel_degree > 1:
            from ..parallel.mp_layers import ColumnParallelLinear, RowParallelLinear
            self.linear1 = ColumnParallelLinear(h, f, weight_attr=_w_attr(cfg), has_bias=True, gather_output=False)
            self.linear2 = RowParallelLinear(f, h, weight_attr=_w_attr(cfg, out_scale), has_bias=True, input_is_parallel=True)
        else:
            self.linear1 = nn.Linear(h, f, weight_attr=_w_attr(cfg))
            self.linear2 = nn.Linear(f, h, weight_attr=_w_attr(cfg, out_scale))

    def forward(self, x, defer_bias=False):
        """defer_bias: return (fc2 output without its bias, the bias), as GPTAttention.forward"""
        if self.cfg.tensor_parallel_degree <= 1:
            from ..ops import mlp as _mlp
            l1, l2 = self.linear1, self.linear2
            if _mlp.available(x._t, l1.weight._t, l1.bias._t, l2.weight._t, l2.bias._t):
                # one node: bias+GELU folded into the GEMM epilogues when that measures faster
                if defer_bias:
                    return _wrap(_mlp.fused_mlp(x._t, l1.weight._t, l1.bias._t, l2.weight._t, None)), l2.bias
                return _wrap(_mlp.fused_mlp(x._t, l1.weight._t, l1.bias._t, l2.weight._t, l2.bias._t))
            if defer_bias:
                h = _cg.matmul_kn(x._t, l1.weight._t)
                h = _ops.bias_gelu(h, l1.bias._t, approximate=True)
                return F.linear(_wrap(h), l2.weight, None), l2.bias
        if self.cfg.tensor_parallel_degree > 1:
            # column-parallel fc1 computed here (bias fused into the GELU): its input must pass
            # c_identity so the backward all-reduces the partial input gradients over the TP group
            from ..parallel.mp_layers import _c_identity
            x = _c_identity(x, self.linear1.model_parallel_group)
        h = _cg.matmul_kn(x._t, self.linear1.weight._t)
        h = _ops.bias_gelu(h, self.linear1.bias._t, approximate=True)
        return self.linear2(_wrap(h))


class GPTDecoderLayer(nn.Layer):
    # stage-3 sharding gathers the whole block as one unit: its forward reads the sublayers'
    # weights directly (fused kernels), so per-sublayer hooks would never fire
    _sharding_unit = True

    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.cfg = cfg
        self.norm1 = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.self_attn = GPTAttention(cfg)
        self.norm2 = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.mlp = GPTMLP(cfg)
        self.dropout = cfg.hidden_dropout

    def _drop(self, t):
        return F.dropout(t, self.dropout, training=self.training) if self.dropout and self.training else t

    def forward(self, x, delta=None, fused=False):
        """fused: (h, m) of forward_fused (the model's residual-deferred chain, called through the
        Layer so forward hooks — stage-3 gathers — fire); else the layer output h + m"""
        h, m = self.forward_fused(x, delta)
        return (h, m) if fused else h + m

    def _add_ln(self, norm, x, delta, dbias=None):
        if delta is None:
            return x, norm(x)
        if norm.weight._t.numel() == 0 and dbias is None:
            # the norm's weights are released by stage-3 sharding (its own unit, outside this
            # block): call it through the Layer so the gather hook fires
            h = x + delta
            return h, norm(h)
        h, y = _ops.fused.add_layer_norm(x._t, delta._t, norm.weight._t, None if norm.bias is None else norm.bias._t,
                                         norm._epsilon, xb=None if dbias is None else dbias._t)
        return _wrap(h), _wrap(y)

    def forward_deferred(self, x, delta, dbias):
        """forward_fused with the output projections' biases deferred too: the layer input is
        ``x + (delta + dbias)``; returns (h, m, mbias). No dropout on the residual branches."""
        h, a_in = self._add_ln(self.norm1, x, delta, dbias)
        a, abias = self.self_attn(a_in, defer_bias=True)
        h2, m_in = self._add_ln(self.norm2, h, a, abias)
        m, mbias = self.mlp(m_in, defer_bias=True)
        return h2, m, mbias

    def forward_fused(self, x, delta):
        """Residual stream with the adds deferred into the next LayerNorm kernel: the layer
        input is ``x + delta`` (delta None = already summed); returns (h, m) whose sum is the
        layer output. Same math as forward(); one pass over the activations fewer per add."""
        h, a_in = self._add_ln(self.norm1, x, delta)
        a = self._drop(self.self_attn(a_in))
        h2, m_in = self._add_ln(self.norm2, h, a)
        return h2, self._drop(self.mlp(m_in))


class GPTEmbeddings(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        if cfg.tensor_parallel_degree > 1:
            from ..parallel.mp_layers import VocabParallelEmbedding
            self.word_embeddings = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, weight_attr=_w_attr(cfg))
        else:
            self.word_embeddings = nn.Embedding(cfg.vocab_size, cfg.hidden_size, weight_attr=_w_attr(cfg))
        self.position_embeddings = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size, weight_attr=_w_attr(cfg))
        self.dropout = cfg.hidden_dropout

    def forward(self, input_ids, position_ids=None):
        S = input_ids._t.shape[-1]
        if position_ids is None:
            position_ids = _wrap(torch.arange(S, device=input_ids._t.device).unsqueeze(0))
        x = self.word_embeddings(input_ids) + self.position_embeddings(position_ids)
        if self.dropout and self.training:
            x = F.dropout(x, self.dropout, training=True)
        return x


class GPTModel(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.cfg = cfg
        self.embeddings = GPTEmbeddings(cfg)
        self.layers = nn.LayerList([GPTDecoderLayer(cfg) for _ in range(cfg.num_layers)])
        self.final_norm = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)

    def _defer_ok(self):
        c = self.cfg
        return (c.tensor_parallel_degree <= 1 and not (c.recompute and self.training)
                and not (c.hidden_dropout and self.training) and os.environ.get("PHA_GPT_DEFER_BIAS", "0") == "1")

    def forward(self, input_ids, position_ids=None):
        x = self.embeddings(input_ids, position_ids)
        delta = None
        if self._defer_ok():
            dbias = None
            for layer in self.layers:
                x, delta, dbias = layer.forward_deferred(x, delta, dbias)
            return self.layers[-1]._add_ln(self.final_norm, x, delta, dbias)[1]
        for layer in self.layers:
            if self.cfg.recompute and self.training:
                from ..parallel.recompute import recompute
                x, delta = recompute(layer, x, delta, fused=True)
            else:
                x, delta = layer(x, delta, fused=True)
        if delta is None:
            return self.final_norm(x)
        return self.layers[-1]._add_ln(self.final_norm, x, delta)[1]


class GPTForPretraining(nn.Layer):
    """Returns per-token logits (or the loss when labels are given)."""

    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.cfg = cfg
        self.gpt = GPTModel(cfg)

    def shared_parameters(self):
        """the tied input / output embedding (read directly by the logits GEMM): stage-3 sharding
        keeps it replicated, as the pipeline form does for its shared layers"""
        return [self.gpt.embeddings.word_embeddings.weight]

    def logits(self, h):
        w = self.gpt.embeddings.word_embeddings.weight
        if self.cfg.tensor_parallel_degree > 1:
            from ..parallel.mp_layers import _c_identity
            h = _c_identity(h)
        return _wrap(_cg.matmul_nt(h._t, w._t))

    def forward(self, input_ids, labels=None, loss_mask=None, position_ids=None):
        h = self.gpt(input_ids, position_ids)
        logits = self.logits(h)
        if labels is None:
            return logits
        return gpt_pretraining_loss(logits, labels, loss_mask, self.cfg.tensor_parallel_degree)


def gpt_pretraining_loss(logits, labels, loss_mask=None, tp_degree=1):
    """GPTPretrainingCriterion: mean CE over masked tokens (fused one-pass HIP CE kernel)."""
    if tp_degree > 1:
        from ..parallel.mp_layers import parallel_cross_entropy
        per_tok = parallel_cross_entropy(logits._t, labels._t)
    else:
        per_tok = _ops.softmax_cross_entropy(logits._t, labels._t)
    if loss_mask is not None:
        m = loss_mask._t.reshape(per_tok.shape).float()
        return _wrap((per_tok * m).sum() / m.sum().clamp_min(1.0))
    return _wrap(per_tok.mean())


# ------------------------------------------------------------------------------ pipeline form
class GPTEmbeddingPipe(GPTEmbeddings):
    """First-stage embedding; the same layer (SharedLayerDesc key "gpt_embed") is rebuilt on the
    last stage as the tied LM head, its weight kept identical by the shared-weight group."""

    @property
    def weight(self):
        return self.word_embeddings.weight

    def forward(self, input_ids):
        return super().forward(input_ids)


def _tied_lm_head(embed, h):
    w = embed.word_embeddings.weight
    if embed.word_embeddings.__class__.__name__ == "VocabParallelEmbedding":
        from ..parallel.mp_layers import _c_identity
        h = _c_identity(h)
    return _wrap(_cg.matmul_nt(h._t, w._t))


class GPTPretrainingCriterionPipe(nn.Layer):
    def __init__(self, tp_degree=1):
        super().__init__()
        self.tp_degree = tp_degree

    def forward(self, logits, labels):
        return gpt_pretraining_loss(logits, labels, None, self.tp_degree)


def _gpt_pipe_descs(cfg):
    from ..parallel.pipeline import LayerDesc, SharedLayerDesc
    descs = [SharedLayerDesc("gpt_embed", GPTEmbeddingPipe, None, "weight", cfg)]
    descs += [LayerDesc(GPTDecoderLayer, cfg) for _ in range(cfg.num_layers)]
    descs += [LayerDesc(nn.LayerNorm, cfg.hidden_size, epsilon=cfg.layer_norm_eps),
              SharedLayerDesc("gpt_embed", GPTEmbeddingPipe, _tied_lm_head, "weight", cfg)]
    return descs


def GPTForPretrainingPipe(cfg: GPTConfig, num_stages=None, topology=None, seg_method="layer:GPTDecoderLayer",
                          recompute_interval=0):
    """GPT pre-training model as a ``PipelineLayer`` (PaddleNLP's GPTForPretrainingPipe layout):
    [embedding] + num_layers x [decoder] + [final LayerNorm, tied LM head], cut at decoder
    layers; loss = GPTPretrainingCriterion on the last stage. Run it under
    ``fleet.distributed_model`` with ``pp_degree`` > 1 (1F1B over RCCL p2p), combinable with TP
    (``cfg.tensor_parallel_degree``) and sharding."""
    from ..parallel.pipeline import PipelineLayer

    class _GPTPipe(PipelineLayer):
        def set_state_dict_from_gpt(self, state):
            """load this stage's slice from a GPTForPretraining state dict (same parameter names as
            the non-pipeline model: gpt.embeddings.*, gpt.layers.{i}.*, gpt.final_norm.*)"""
            import numpy as np
            for i in range(self._start, self._end):
                if i == 0 or i == len(self._layers_desc) - 1:
                    prefix = "gpt.embeddings."
                elif i == len(self._layers_desc) - 2:
                    prefix = "gpt.final_norm."
                else:
                    prefix = f"gpt.layers.{i - 1}."
                layer = self._built[i - self._start]   # every desc builds (or reuses) one layer
                for name, prm in layer.named_parameters():
                    v = state[prefix + name]
                    prm.set_value(v.numpy() if hasattr(v, "numpy") else np.asarray(v))

    return _GPTPipe(_gpt_pipe_descs(cfg), num_stages=num_stages, topology=topology,
                    loss_fn=GPTPretrainingCriterionPipe(cfg.tensor_parallel_degree), seg_method=seg_method,
                    recompute_interval=recompute_interval)


def gpt_1_3b(**kw):
    return GPTForPretraining(gpt_config("gpt3-1.3b", **kw))
