"""Fused transformer layers (reference: python/paddle/incubate/nn/layer/fused_transformer.py,
fused_linear.py). Parameter shapes match the reference so checkpoints interchange."""
from __future__ import annotations

from ...nn.layer.layers import Layer
from ...nn import initializer as I
from . import functional  # noqa: F401
from . import functional as FF

__all__ = ["FusedMultiHeadAttention", "FusedFeedForward", "FusedTransformerEncoderLayer", "FusedMultiTransformer",
           "FusedLinear", "FusedBiasDropoutResidualLayerNorm"]


class FusedLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, transpose_weight=False,
                 name=None):
        super().__init__()
        shape = [out_features, in_features] if transpose_weight else [in_features, out_features]
        self.weight = self.create_parameter(shape, attr=weight_attr)
        self.bias = self.create_parameter([out_features], attr=bias_attr, is_bias=True)
        self.transpose_weight = transpose_weight

    def forward(self, input):
        return FF.fused_linear(input, self.weight, self.bias, self.transpose_weight)


class FusedBiasDropoutResidualLayerNorm(Layer):
    def __init__(self, embed_dim, dropout_rate=0.5, weight_attr=None, bias_attr=None, epsilon=1e-5, name=None):
        super().__init__()
        self.embed_dim, self.dropout_rate, self._epsilon = embed_dim, dropout_rate, epsilon
        self.linear_bias = self.create_parameter([embed_dim], attr=bias_attr, is_bias=True)
        self.ln_scale = self.create_parameter([embed_dim], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.ln_bias = self.create_parameter([embed_dim], attr=bias_attr, is_bias=True)

    def forward(self, x, residual):
        return FF.fused_bias_dropout_residual_layer_norm(x, residual, self.linear_bias, self.ln_scale, self.ln_bias,
                                                         self.dropout_rate, self._epsilon, self.training)


class FusedMultiHeadAttention(Layer):
    def __init__(self, embed_dim, num_heads, dropout_rate=0.5, attn_dropout_rate=0.5, kdim=None, vdim=None,
                 normalize_before=False, need_weights=False, qkv_weight_attr=None, qkv_bias_attr=None,
                 linear_weight_attr=None, linear_bias_attr=None, pre_ln_scale_attr=None, pre_ln_bias_attr=None,
                 ln_scale_attr=None, ln_bias_attr=None, epsilon=1e-5, nranks=1, ring_id=-1, name=None):
        super().__init__()
        if embed_dim % num_heads != 0:
            raise ValueError("embed_dim must be divisible by num_heads")
        if need_weights:
            raise ValueError("need_weights=True is not supported by the fused attention")
        self.embed_dim, self.normalize_before, self._epsilon = embed_dim, normalize_before, epsilon
        self.dropout_rate, self.attn_dropout_rate, self._ring_id = dropout_rate, attn_dropout_rate, ring_id
        self.num_heads = num_heads // nranks
        self.head_dim = embed_dim // num_heads
        self.qkv_weight = self.create_parameter([3, self.num_heads, self.head_dim, embed_dim], attr=qkv_weight_attr)
        self.qkv_bias = self.create_parameter([3, self.num_heads, self.head_dim], attr=qkv_bias_attr, is_bias=True)
        self.linear_weight = self.create_parameter([self.num_heads * self.head_dim, embed_dim],
                                                   attr=linear_weight_attr)
        self.linear_bias = self.create_parameter([embed_dim], attr=linear_bias_attr, is_bias=True)
        if normalize_before:
            self.pre_ln_scale = self.create_parameter([embed_dim], attr=pre_ln_scale_attr,
                                                      default_initializer=I.Constant(1.0))
            self.pre_ln_bias = self.create_parameter([embed_dim], attr=pre_ln_bias_attr, is_bias=True)
            self.ln_scale = self.ln_bias = None
        else:
            self.pre_ln_scale = self.pre_ln_bias = None
            self.ln_scale = self.create_parameter([embed_dim], attr=ln_scale_attr, default_initializer=I.Constant(1.0))
            self.ln_bias = self.create_parameter([embed_dim], attr=ln_bias_attr, is_bias=True)

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        return FF.fused_multi_head_attention(
            query, self.qkv_weight, self.linear_weight, self.normalize_before, self.pre_ln_scale, self.pre_ln_bias,
            self.ln_scale, self.ln_bias, self._epsilon, self.qkv_bias, self.linear_bias, cache, attn_mask,
            self.dropout_rate, self.attn_dropout_rate, self._epsilon, self.training, "upscale_in_train", self._ring_id)


class FusedFeedForward(Layer):
    def __init__(self, d_model, dim_feedforward, dropout_rate=0.1, epsilon=1e-05, activation="relu",
                 act_dropout_rate=None, normalize_before=False, linear1_weight_attr=None, linear1_bias_attr=None,
                 linear2_weight_attr=None, linear2_bias_attr=None, ln1_scale_attr=None, ln1_bias_attr=None,
                 ln2_scale_attr=None, ln2_bias_attr=None, nranks=1, ring_id=-1, name=None):
        super().__init__()
        self._d_model, self._epsilon, self._act = d_model, epsilon, activation
        self._dropout_rate = dropout_rate
        self._act_dropout_rate = dropout_rate if act_dropout_rate is None else act_dropout_rate
        self._normalize_before, self._ring_id = normalize_before, ring_id
        dff = dim_feedforward // nranks
        self._linear1_weight = self.create_parameter([d_model, dff], attr=linear1_weight_attr)
        self._linear1_bias = self.create_parameter([dff], attr=linear1_bias_attr, is_bias=True)
        self._linear2_weight = self.create_parameter([dff, d_model], attr=linear2_weight_attr)
        self._linear2_bias = self.create_parameter([d_model], attr=linear2_bias_attr, is_bias=True)
        if normalize_before:
            self._ln1_scale = self.create_parameter([d_model], attr=ln1_scale_attr, default_initializer=I.Constant(1.0))
            self._ln1_bias = self.create_parameter([d_model], attr=ln1_bias_attr, is_bias=True)
            self._ln2_scale = self._ln2_bias = None
        else:
            self._ln1_scale = self._ln1_bias = None
            self._ln2_scale = self.create_parameter([d_model], attr=ln2_scale_attr, default_initializer=I.Constant(1.0))
            self._ln2_bias = self.create_parameter([d_model], attr=ln2_bias_attr, is_bias=True)

    def forward(self, src, cache=None):
        return FF.fused_feedforward(src, self._linear1_weight, self._linear2_weight, self._linear1_bias,
                                    self._linear2_bias, self._ln1_scale, self._ln1_bias, self._ln2_scale,
                                    self._ln2_bias, self._act_dropout_rate, self._dropout_rate, self._act,
                                    self._epsilon, self._epsilon, self._normalize_before, self.training,
                                    ring_id=self._ring_id)


class FusedTransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout_rate=0.1, activation="relu", attn_dropout_rate=None,
                 act_dropout_rate=None, normalize_before=False, weight_attr=None, bias_attr=None):
        super().__init__()
        attn_dropout_rate = dropout_rate if attn_dropout_rate is None else attn_dropout_rate
        act_dropout_rate = dropout_rate if act_dropout_rate is None else act_dropout_rate
        self.normalize_before = normalize_before
        self.fused_attn = FusedMultiHeadAttention(d_model, nhead, dropout_rate=dropout_rate,
                                                  attn_dropout_rate=attn_dropout_rate,
                                                  normalize_before=normalize_before, qkv_weight_attr=weight_attr,
                                                  qkv_bias_attr=bias_attr, linear_weight_attr=weight_attr,
                                                  linear_bias_attr=bias_attr)
        self.ffn = FusedFeedForward(d_model, dim_feedforward, dropout_rate=dropout_rate, activation=activation,
                                    act_dropout_rate=act_dropout_rate, normalize_before=normalize_before,
                                    linear1_weight_attr=weight_attr, linear1_bias_attr=bias_attr,
                                    linear2_weight_attr=weight_attr, linear2_bias_attr=bias_attr)

    def forward(self, src, src_mask=None, cache=None):
        if cache is None:
            return self.ffn(self.fused_attn(src, attn_mask=src_mask))
        out, new_cache = self.fused_attn(src, attn_mask=src_mask, cache=cache)
        return self.ffn(out), new_cache


class FusedMultiTransformer(Layer):
    """Decoder stack for generation with in-place KV caches (see functional.fused_multi_transformer)."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, ln_scale_attrs=None, ln_bias_attrs=None, qkv_weight_attrs=None,
                 qkv_bias_attrs=None, linear_weight_attrs=None, linear_bias_attrs=None, ffn_ln_scale_attrs=None,
                 ffn_ln_bias_attrs=None, ffn1_weight_attrs=None, ffn1_bias_attrs=None, ffn2_weight_attrs=None,
                 ffn2_bias_attrs=None, epsilon=1e-5, num_layers=-1, nranks=1, trans_qkvw=True, ring_id=-1, name=None):
        super().__init__()
        if num_layers < 0:
            num_layers = len(qkv_weight_attrs) if isinstance(qkv_weight_attrs, (list, tuple)) else 1
        self.normalize_before, self._epsilon, self._act = normalize_before, epsilon, activation
        self._dropout_rate, self._trans_qkvw, self._ring_id = dropout_rate, trans_qkvw, ring_id
        self.num_heads = num_heads // nranks
        self.head_dim = embed_dim // num_heads
        dff = dim_feedforward // nranks

        def attr(a, i):
            return a[i] if isinstance(a, (list, tuple)) else a

        from ...nn.layer.container import ParameterList
        names = ["ln_scales", "ln_biases", "qkv_weights", "qkv_biases", "linear_weights", "linear_biases",
                 "ffn_ln_scales", "ffn_ln_biases", "ffn1_weights", "ffn1_biases", "ffn2_weights", "ffn2_biases"]
        lists = {n: [] for n in names}
        H, D = self.num_heads, self.head_dim
        for i in range(num_layers):
            lists["ln_scales"].append(self.create_parameter([embed_dim], attr=attr(ln_scale_attrs, i),
                                                            default_initializer=I.Constant(1.0)))
            lists["ln_biases"].append(self.create_parameter([embed_dim], attr=attr(ln_bias_attrs, i), is_bias=True))
            qshape = [3, H, D, embed_dim] if trans_qkvw else [embed_dim, 3, H, D]
            lists["qkv_weights"].append(self.create_parameter(qshape, attr=attr(qkv_weight_attrs, i)))
            lists["qkv_biases"].append(self.create_parameter([3, H, D], attr=attr(qkv_bias_attrs, i), is_bias=True))
            lists["linear_weights"].append(self.create_parameter([H * D, embed_dim], attr=attr(linear_weight_attrs, i)))
            lists["linear_biases"].append(self.create_parameter([embed_dim], attr=attr(linear_bias_attrs, i),
                                                                is_bias=True))
            lists["ffn_ln_scales"].append(self.create_parameter([embed_dim], attr=attr(ffn_ln_scale_attrs, i),
                                                                default_initializer=I.Constant(1.0)))
            lists["ffn_ln_biases"].append(self.create_parameter([embed_dim], attr=attr(ffn_ln_bias_attrs, i),
                                                                is_bias=True))
            lists["ffn1_weights"].append(self.create_parameter([embed_dim, dff], attr=attr(ffn1_weight_attrs, i)))
            lists["ffn1_biases"].append(self.create_parameter([dff], attr=attr(ffn1_bias_attrs, i), is_bias=True))
            lists["ffn2_weights"].append(self.create_parameter([dff, embed_dim], attr=attr(ffn2_weight_attrs, i)))
            lists["ffn2_biases"].append(self.create_parameter([embed_dim], attr=attr(ffn2_bias_attrs, i),
                                                              is_bias=True))
        for n in names:
            setattr(self, n, ParameterList(lists[n]))

    def forward(self, src, attn_mask=None, caches=None, time_step=None):
        L = lambda n: list(getattr(self, n))  # noqa: E731
        return FF.fused_multi_transformer(
            src, L("ln_scales"), L("ln_biases"), L("qkv_weights"), L("qkv_biases"), L("linear_weights"),
            L("linear_biases"), L("ffn_ln_scales"), L("ffn_ln_biases"), L("ffn1_weights"), L("ffn1_biases"),
            L("ffn2_weights"), L("ffn2_biases"), self.normalize_before, self._epsilon, caches, time_step, attn_mask,
            self._dropout_rate, self._act, self.training, "upscale_in_train", self._trans_qkvw, self._ring_id)
