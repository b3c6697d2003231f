"""BERT (base/large) for pre-training — the model of the BASELINE "BERT-base bf16 seq512,
fleet DP" config (reference usage: the fleet/ dygraph BERT tests, e.g.
python/paddle/fluid/tests/unittests/dygraph_to_static/bert_dygraph_model.py, whose
structure — embeddings(word+pos+type) → post-LN encoder → pooler, MLM head tied to the word
embeddings + NSP head — this follows; parameter layout PaddleNLP-style).

MI355X-first choices: fused QKV GEMM; unmasked attention on the MFMA flash-attention
kernel (padded batches / attention dropout use the fused SDPA path); bias-GELU and
LayerNorm on the HIP kernels; the MLM loss on the one-pass softmax-CE kernel over only the
masked positions (gathered first, so the vocab GEMM runs on ~15 % of the tokens).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as TF

from ..framework.core import Tensor, _wrap
from .. import nn
from ..nn import functional as F
from ..nn import initializer as I
from .. import ops as _ops

__all__ = ["BertConfig", "BertModel", "BertForPretraining", "BertPretrainingCriterion", "bert_config",
           "BERT_CONFIGS"]


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_layers: int = 12
    num_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.1
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0

    @property
    def head_dim(self):
        return self.hidden_size // self.num_heads


BERT_CONFIGS = {
    "bert-base": dict(),
    "bert-large": dict(hidden_size=1024, num_layers=24, num_heads=16, intermediate_size=4096),
    "bert-tiny": dict(vocab_size=512, hidden_size=64, num_layers=2, num_heads=4, intermediate_size=256,
                      max_position_embeddings=128),
}


def bert_config(name, **overrides):
    d = dict(BERT_CONFIGS[name])
    d.update(overrides)
    return BertConfig(**d)


def _attr(cfg):
    return nn.ParamAttr(initializer=I.TruncatedNormal(0.0, cfg.initializer_range))


class BertEmbeddings(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.word_embeddings = nn.Embedding(cfg.vocab_size, cfg.hidden_size, weight_attr=_attr(cfg))
        self.position_embeddings = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size, weight_attr=_attr(cfg))
        self.token_type_embeddings = nn.Embedding(cfg.type_vocab_size, cfg.hidden_size, weight_attr=_attr(cfg))
        self.layer_norm = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.dropout = cfg.hidden_dropout

    def forward(self, input_ids, token_type_ids=None, position_ids=None):
        S = input_ids.shape[-1]
        dev = input_ids._t.device
        if position_ids is None:
            position_ids = _wrap(torch.arange(S, device=dev).unsqueeze(0))
        if token_type_ids is None:
            token_type_ids = _wrap(torch.zeros_like(input_ids._t))
        x = (self.word_embeddings(input_ids) + self.position_embeddings(position_ids)
             + self.token_type_embeddings(token_type_ids))
        x = self.layer_norm(x)
        return F.dropout(x, self.dropout, training=self.training) if self.dropout else x


class BertSelfAttention(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.qkv = nn.Linear(cfg.hidden_size, 3 * cfg.hidden_size, weight_attr=_attr(cfg))
        self.out = nn.Linear(cfg.hidden_size, cfg.hidden_size, weight_attr=_attr(cfg))

    def forward(self, x, attn_bias=None):
        B, S, _ = x.shape
        Hn, Dh = self.cfg.num_heads, self.cfg.head_dim
        qkv = self.qkv(x)._t.reshape(B, S, Hn, 3 * Dh)
        drop = self.cfg.attention_dropout if self.training else 0.0
        # padded batch: additive key mask [B, 1, 1, S]; attention dropout in-kernel; the packed
        # entry writes dq | dk | dv into one gradient (no split-backward concatenation)
        o = _ops.flash_attention_qkvpacked(qkv, Hn, causal=False, dropout_p=drop, training=self.training,
                                           mask=attn_bias)
        return self.out(_wrap(o.reshape(B, S, Hn * Dh)))


class BertLayer(nn.Layer):
    """Post-LN: x = LN(x + Attn(x)); x = LN(x + FFN(x))."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.attention = BertSelfAttention(cfg)
        self.norm1 = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.linear1 = nn.Linear(cfg.hidden_size, cfg.intermediate_size, weight_attr=_attr(cfg))
        self.linear2 = nn.Linear(cfg.intermediate_size, cfg.hidden_size, weight_attr=_attr(cfg))
        self.norm2 = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)

    def _drop(self, t):
        p = self.cfg.hidden_dropout
        return F.dropout(t, p, training=self.training) if p and self.training else t

    def _add_norm(self, y, x, norm):
        """LN(x + dropout(y)) as one fused bias-dropout-residual-LayerNorm pass each way"""
        p = self.cfg.hidden_dropout if self.training else 0.0
        yt, xt = y._t, x._t
        return _wrap(_ops.bias_dropout_residual_layer_norm(yt.contiguous(), xt.contiguous().to(yt.dtype), None,
                                                          norm.weight._t, norm.bias._t, p, self.training,
                                                          norm._epsilon))

    def forward(self, x, attn_bias=None):
        x = self._add_norm(self.attention(x, attn_bias), x, self.norm1)
        from ..ops import mlp as _mlp
        l1, l2 = self.linear1, self.linear2
        if _mlp.available(x._t, l1.weight._t, l1.bias._t, l2.weight._t, l2.bias._t):
            # one autograd node: both weight gradients on the own TN kernel with the bias gradients
            # from its B fragments, the exact-GELU backward pass without a column-sum side job
            y = _wrap(_mlp.fused_mlp(x._t, l1.weight._t, l1.bias._t, l2.weight._t, l2.bias._t, approximate=False))
            return self._add_norm(y, x, self.norm2)
        h = torch.matmul(x._t, self.linear1.weight._t)
        h = _ops.bias_gelu(h, self.linear1.bias._t, approximate=False)
        return self._add_norm(self.linear2(_wrap(h)), x, self.norm2)


class BertModel(nn.Layer):
    def __init__(self, cfg: BertConfig):
        super().__init__()
        self.cfg = cfg
        self.embeddings = BertEmbeddings(cfg)
        self.layers = nn.LayerList([BertLayer(cfg) for _ in range(cfg.num_layers)])
        self.pooler = nn.Linear(cfg.hidden_size, cfg.hidden_size, weight_attr=_attr(cfg))

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None):
        attn_bias = None
        if attention_mask is not None:
            m = attention_mask._t if isinstance(attention_mask, Tensor) else attention_mask
            attn_bias = ((1.0 - m.float()) * -1e4).reshape(m.shape[0], 1, 1, m.shape[-1])
        x = self.embeddings(input_ids, token_type_ids, position_ids)
        for layer in self.layers:
            x = layer(x, attn_bias)
        pooled = F.tanh(self.pooler(_wrap(x._t[:, 0])))
        return x, pooled


class BertForPretraining(nn.Layer):
    """MLM (tied decoder) + NSP heads. ``masked_positions``: flat indices into [B*S] of the
    masked tokens; the vocab projection runs only on those rows."""

    def __init__(self, cfg: BertConfig):
        super().__init__()
        self.cfg = cfg
        self.bert = BertModel(cfg)
        self.transform = nn.Linear(cfg.hidden_size, cfg.hidden_size, weight_attr=_attr(cfg))
        self.transform_norm = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.decoder_bias = self.create_parameter([cfg.vocab_size], is_bias=True)
        self.nsp = nn.Linear(cfg.hidden_size, 2, weight_attr=_attr(cfg))

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None,
                masked_positions=None):
        seq, pooled = self.bert(input_ids, token_type_ids, position_ids, attention_mask)
        h = seq._t.reshape(-1, seq.shape[-1])
        if masked_positions is not None:
            mp = masked_positions._t if isinstance(masked_positions, Tensor) else masked_positions
            h = h.index_select(0, mp.reshape(-1).long())
        t = self.transform(_wrap(h))._t
        t = self.transform_norm(_wrap(_ops.gelu(t.contiguous(), approximate=False)))._t
        w = self.bert.embeddings.word_embeddings.weight._t
        logits = torch.matmul(t, w.t()) + self.decoder_bias._t
        return _wrap(logits), self.nsp(pooled)


class BertPretrainingCriterion(nn.Layer):
    def __init__(self, vocab_size):
        super().__init__()
        self.vocab_size = vocab_size

    def forward(self, mlm_logits, nsp_logits, mlm_labels, nsp_labels):
        mlm = _ops.softmax_cross_entropy(mlm_logits._t.contiguous(), mlm_labels._t.reshape(-1).long())
        if mlm.dim():   # mean over the labelled positions, as a masked sum (boolean indexing syncs the host)
            valid = (mlm_labels._t.reshape(-1) != -100).to(torch.float32)
            mlm = (mlm.float() * valid).sum() / valid.sum().clamp_min(1.0)
        nsp = TF.cross_entropy(nsp_logits._t.float(), nsp_labels._t.reshape(-1).long())
        return _wrap(mlm + nsp)
