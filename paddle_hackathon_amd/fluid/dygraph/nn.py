"""``fluid.dygraph.nn`` layers with the 1.x constructor signatures (reference:
python/paddle/fluid/dygraph/nn.py): they hold their parameters and call the framework's
functional ops (own HIP kernels where those exist, e.g. conv / norm / linear)."""
from __future__ import annotations

import numpy as np
import torch

from ...nn.layer.layers import Layer
from ...nn import functional as F
from ...nn import initializer as I
from ...nn.layer.conv_norm_pool import BatchNorm, SpectralNorm as _SN  # noqa: F401
from ...framework.core import _wrap
from ..layers._common import T, W, act as _act
from ..layers import nn as LN

__all__ = ["Conv2D", "Conv3D", "Pool2D", "Linear", "BatchNorm", "Dropout", "Embedding", "GRUUnit", "InstanceNorm",
           "LayerNorm", "NCE", "PRelu", "BilinearTensorProduct", "Conv2DTranspose", "Conv3DTranspose", "GroupNorm",
           "SpectralNorm", "TreeConv", "Flatten"]


def _nt(v, n):
    return list(v) if isinstance(v, (list, tuple)) else [v] * n


class _ConvND(Layer):
    def __init__(self, nd, transpose, num_channels, num_filters, filter_size, stride, padding, dilation, groups,
                 param_attr, bias_attr, act, dtype, output_size=None):
        super().__init__()
        self._nd, self._transpose = nd, transpose
        self._groups = groups or 1
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._act, self._output_size = act, output_size
        k = _nt(filter_size, nd)
        if transpose:
            shape = [num_channels, num_filters // self._groups] + k
        else:
            shape = [num_filters, num_channels // self._groups] + k
        fan_in = (num_channels // self._groups) * int(np.prod(k))
        self.weight = self.create_parameter(shape, param_attr, dtype,
                                            default_initializer=I.Normal(0.0, (2.0 / fan_in) ** 0.5))
        self.bias = None if bias_attr is False else self.create_parameter([num_filters], bias_attr, dtype,
                                                                          is_bias=True)

    def forward(self, input):
        if self._transpose:
            f = F.conv2d_transpose if self._nd == 2 else F.conv3d_transpose
            y = f(input, self.weight, self.bias, self._stride, self._padding, 0, self._dilation, self._groups,
                  self._output_size) if self._nd == 2 else \
                f(input, self.weight, self.bias, self._stride, self._padding, 0, self._groups, self._dilation,
                  self._output_size)
        else:
            f = F.conv2d if self._nd == 2 else F.conv3d
            y = f(input, self.weight, self.bias, self._stride, self._padding, self._dilation, self._groups)
        return _act(y, self._act)


class Conv2D(_ConvND):
    def __init__(self, num_channels, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,
                 param_attr=None, bias_attr=None, use_cudnn=True, act=None, dtype="float32"):
        super().__init__(2, False, num_channels, num_filters, filter_size, stride, padding, dilation, groups,
                         param_attr, bias_attr, act, dtype)


class Conv3D(_ConvND):
    def __init__(self, num_channels, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,
                 param_attr=None, bias_attr=None, use_cudnn=True, act=None, dtype="float32"):
        super().__init__(3, False, num_channels, num_filters, filter_size, stride, padding, dilation, groups,
                         param_attr, bias_attr, act, dtype)


class Conv2DTranspose(_ConvND):
    def __init__(self, num_channels, num_filters, filter_size, output_size=None, padding=0, stride=1, dilation=1,
                 groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, dtype="float32"):
        super().__init__(2, True, num_channels, num_filters, filter_size, stride, padding, dilation, groups,
                         param_attr, bias_attr, act, dtype, output_size)


class Conv3DTranspose(_ConvND):
    def __init__(self, num_channels, num_filters, filter_size, output_size=None, padding=0, stride=1, dilation=1,
                 groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, dtype="float32"):
        super().__init__(3, True, num_channels, num_filters, filter_size, stride, padding, dilation, groups,
                         param_attr, bias_attr, act, dtype, output_size)


class Pool2D(Layer):
    def __init__(self, pool_size=-1, pool_type="max", pool_stride=1, pool_padding=0, global_pooling=False,
                 use_cudnn=True, ceil_mode=False, exclusive=True, data_format="NCHW"):
        super().__init__()
        self._args = (pool_size, pool_type, pool_stride, pool_padding, global_pooling, use_cudnn, ceil_mode, None,
                      exclusive, data_format)

    def forward(self, input):
        return LN.pool2d(input, *self._args)


class Linear(Layer):
    def __init__(self, input_dim, output_dim, param_attr=None, bias_attr=None, act=None, dtype="float32"):
        super().__init__()
        self._act = act
        self.weight = self.create_parameter([input_dim, output_dim], param_attr, dtype)
        self.bias = None if bias_attr is False else self.create_parameter([output_dim], bias_attr, dtype,
                                                                          is_bias=True)

    def forward(self, input):
        return _act(F.linear(input, self.weight, self.bias), self._act)


class Dropout(Layer):
    def __init__(self, p=0.5, seed=None, dropout_implementation="downgrade_in_infer", is_test=False):
        super().__init__()
        self._p, self._seed, self._impl, self._is_test = p, seed, dropout_implementation, is_test

    def forward(self, input):
        return LN.dropout(input, self._p, is_test=not self.training or self._is_test, seed=self._seed,
                          dropout_implementation=self._impl)


class Embedding(Layer):
    """lookup_table_v2: output = ids.shape + [emb_dim]"""

    def __init__(self, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None,
                 dtype="float32"):
        super().__init__()
        self._size = list(size)
        self._padding_idx = None if padding_idx is None else (padding_idx if padding_idx >= 0 else
                                                              padding_idx + size[0])
        self.weight = self.create_parameter(self._size, param_attr, dtype, default_initializer=I.XavierUniform())

    def forward(self, input):
        return F.embedding(input, self.weight, self._padding_idx)


class GRUUnit(Layer):
    def __init__(self, size, param_attr=None, bias_attr=None, activation="tanh", gate_activation="sigmoid",
                 origin_mode=False, dtype="float32"):
        super().__init__()
        H = size // 3
        self._H, self._act, self._gact, self._origin = H, activation, gate_activation, origin_mode
        self.weight = self.create_parameter([H, 3 * H], param_attr, dtype)
        self.bias = None if bias_attr is False else self.create_parameter([1, 3 * H], bias_attr, dtype, is_bias=True)

    def forward(self, input, hidden):
        from ..layers.rnn import _act as ract
        H = self._H
        x, h = T(input), T(hidden)
        wt = T(self.weight)
        if self.bias is not None:
            x = x + T(self.bias)
        xu, xr, xc = x.split(H, -1)
        u = ract(self._gact)(xu + h @ wt[:, :H])
        r = ract(self._gact)(xr + h @ wt[:, H:2 * H])
        rh = r * h
        c = ract(self._act)(xc + rh @ wt[:, 2 * H:])
        hn = u * h + (1 - u) * c if self._origin else (1 - u) * h + u * c
        return W(hn), W(rh), W(torch.cat([u, r, c], -1))


class InstanceNorm(Layer):
    def __init__(self, num_channels, epsilon=1e-5, param_attr=None, bias_attr=None, dtype="float32"):
        super().__init__()
        self._eps = epsilon
        self.scale = None if param_attr is False else self.create_parameter([num_channels], param_attr, dtype,
                                                                            default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([num_channels], bias_attr, dtype,
                                                                          is_bias=True)

    def forward(self, input):
        return F.instance_norm(input, weight=self.scale, bias=self.bias, eps=self._eps)


class LayerNorm(Layer):
    def __init__(self, normalized_shape, scale=True, shift=True, epsilon=1e-05, param_attr=None, bias_attr=None,
                 act=None, dtype="float32"):
        super().__init__()
        self._shape = [normalized_shape] if isinstance(normalized_shape, int) else list(normalized_shape)
        self._eps, self._act = epsilon, act
        n = int(np.prod(self._shape))
        self.weight = self.create_parameter([n], param_attr, dtype, default_initializer=I.Constant(1.0)) \
            if scale else None
        self.bias = self.create_parameter([n], bias_attr, dtype, is_bias=True) if shift else None

    def forward(self, input):
        return _act(F.layer_norm(input, self._shape, self.weight, self.bias, self._eps), self._act)


class GroupNorm(Layer):
    def __init__(self, channels, groups, epsilon=1e-05, param_attr=None, bias_attr=None, act=None,
                 data_layout="NCHW", dtype="float32"):
        super().__init__()
        self._groups, self._eps, self._act, self._layout = groups, epsilon, act, data_layout
        self.weight = self.create_parameter([channels], param_attr, dtype, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([channels], bias_attr, dtype, is_bias=True)

    def forward(self, input):
        return _act(F.group_norm(input, self._groups, self._eps, self.weight, self.bias, self._layout), self._act)


class SpectralNorm(_SN):
    pass


class NCE(Layer):
    """noise-contrastive estimation loss with uniform / log-uniform / custom negative sampling"""

    def __init__(self, num_total_classes, dim, sample_weight=None, param_attr=None, bias_attr=None,
                 num_neg_samples=None, sampler="uniform", custom_dist=None, seed=0, is_sparse=False,
                 dtype="float32"):
        super().__init__()
        self._C, self._neg = num_total_classes, num_neg_samples or 10
        self._sampler, self._custom = sampler, custom_dist
        self._gen = torch.Generator()
        self._gen.manual_seed(int(seed) if seed else 0)
        self.weight = self.create_parameter([num_total_classes, dim], param_attr, dtype)
        self.bias = None if bias_attr is False else self.create_parameter([num_total_classes, 1], bias_attr, dtype,
                                                                          is_bias=True)

    def _probs(self):
        C = self._C
        if self._sampler == "custom_dist":
            return torch.as_tensor(np.asarray(self._custom), dtype=torch.float64)
        if self._sampler == "log_uniform":
            k = torch.arange(C, dtype=torch.float64)
            return torch.log((k + 2) / (k + 1)) / np.log(C + 1)
        return torch.full((C,), 1.0 / C, dtype=torch.float64)

    def forward(self, input, label, sample_weight=None):
        x = T(input)
        y = T(label).reshape(x.shape[0], -1).long()
        q = self._probs()
        neg = torch.multinomial(q, self._neg, replacement=True, generator=self._gen).to(x.device)
        wt = T(self.weight)

        def logit(ids):
            s = (x[:, None, :] * wt[ids]).sum(-1) if ids.dim() == 2 else x @ wt[ids].t()
            if self.bias is not None:
                s = s + (T(self.bias)[ids, 0] if ids.dim() == 2 else T(self.bias)[ids, 0][None])
            return s
        qd = q.to(x.device, x.dtype)
        k = float(self._neg)
        s_pos = logit(y)
        s_neg = logit(neg)
        p_pos = torch.sigmoid(s_pos - torch.log(k * qd[y]))
        p_neg = torch.sigmoid(s_neg - torch.log(k * qd[neg])[None])
        cost = -(torch.log(p_pos + 1e-20).sum(1) + torch.log(1 - p_neg + 1e-20).sum(1))
        if sample_weight is not None:
            cost = cost * T(sample_weight).reshape(-1)
        return W(cost[:, None])


class PRelu(Layer):
    def __init__(self, mode, channel=None, input_shape=None, param_attr=None, dtype="float32"):
        super().__init__()
        self._mode = mode
        if mode == "all":
            shape = [1]
        elif mode == "channel":
            shape = [1, channel, 1, 1]
        else:
            shape = [1] + list(input_shape[1:])
        self.weight = self.create_parameter(shape, param_attr, dtype, default_initializer=I.Constant(0.25))

    def forward(self, input):
        x, a = T(input), T(self.weight)
        if self._mode == "channel" and x.dim() != 4:
            a = a.reshape([1, -1] + [1] * (x.dim() - 2))
        return W(torch.where(x > 0, x, a * x))


class BilinearTensorProduct(Layer):
    def __init__(self, input1_dim, input2_dim, output_dim, name=None, act=None, param_attr=None, bias_attr=None,
                 dtype="float32"):
        super().__init__()
        self._act = act
        self.weight = self.create_parameter([output_dim, input1_dim, input2_dim], param_attr, dtype)
        self.bias = None if bias_attr is False else self.create_parameter([1, output_dim], bias_attr, dtype,
                                                                          is_bias=True)

    def forward(self, x, y):
        return _act(F.bilinear(x, y, self.weight, self.bias), self._act)


def _tree_patches(edges, max_depth):
    """continuous-binary-tree patches (tree2col.cc): per root node, (node, eta_l, eta_r, eta_t)"""
    node_count = 0
    for u, v in edges:
        if u != 0 and v != 0:
            node_count += 1
    node_count += 1
    tr = [[] for _ in range(node_count + 1)]
    for u, v in edges:
        if u != 0 and v != 0:
            tr[u].append(v)
        else:
            break
    md = float(max_depth)
    patches = []
    for root in range(1, node_count + 1):
        stack = [(root, 1, 1, 0)]
        patch = [(root, 1, 1, 0)]
        visited = {root}
        while stack:
            node, _, _, depth = stack[-1]
            end = True
            sz = len(tr[node])
            for i, v in enumerate(tr[node]):
                if v not in visited and depth + 1 < max_depth:
                    visited.add(v)
                    stack.append((v, i, sz, depth + 1))
                    patch.append((v, i + 1, sz, depth + 1))
                    end = False
            if end:
                stack.pop()
        rows = []
        for node, index, pclen, depth in patch:
            eta_t = (md - depth) / md
            temp = 0.5 if pclen == 1 else (index - 1.0) / (pclen - 1.0)
            eta_l = (1.0 - eta_t) * temp
            eta_r = (1.0 - eta_t) * (1.0 - eta_l)
            rows.append((node - 1, eta_l, eta_r, eta_t))
        patches.append(rows)
    return patches


class TreeConv(Layer):
    """tree-based convolution (TBCNN, tree_conv_op.h): each node's patch mixes its subtree (to
    ``max_depth``) with left / right / top weights; out [B, N, output_size, num_filters]"""

    def __init__(self, feature_size, output_size, num_filters=1, max_depth=2, act="tanh", param_attr=None,
                 bias_attr=None, name=None, dtype="float32"):
        super().__init__()
        self._F, self._out, self._nf, self._depth, self._act = feature_size, output_size, num_filters, max_depth, act
        self.weight = self.create_parameter([feature_size, 3, output_size, num_filters], param_attr, dtype)
        self.bias = None if bias_attr is False else self.create_parameter([1, num_filters], bias_attr, dtype,
                                                                          is_bias=True)

    def forward(self, nodes_vector, edge_set):
        x = T(nodes_vector)
        e = T(edge_set).long().cpu().tolist()
        B, N, Fd = x.shape
        wt = T(self.weight).reshape(Fd * 3, self._out * self._nf)
        outs = []
        for b in range(B):
            patches = _tree_patches(e[b], self._depth)
            P = torch.zeros(N, Fd * 3, dtype=x.dtype, device=x.device)
            rows = []
            for k, patch in enumerate(patches[:N]):
                coef = torch.zeros(N, 3, dtype=x.dtype, device=x.device)
                for node, el, er, et in patch:
                    coef[node, 0] += el
                    coef[node, 1] += er
                    coef[node, 2] += et
                rows.append((coef.t() @ x[b]).t().reshape(-1))     # [F*3] laid out f*3 + {l,r,t}
            if rows:
                P = torch.cat([torch.stack(rows), P[len(rows):]], 0)
            outs.append((P @ wt).reshape(N, self._out, self._nf))
        y = torch.stack(outs)
        if self.bias is not None:
            y = y + T(self.bias).reshape(1, 1, 1, -1)
        return _act(W(y), self._act)


class Flatten(Layer):
    def __init__(self, start_axis=1, stop_axis=-1):
        super().__init__()
        self._a, self._b = start_axis, stop_axis

    def forward(self, input):
        return _wrap(torch.flatten(T(input), self._a, self._b))
