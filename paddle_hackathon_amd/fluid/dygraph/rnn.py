"""``fluid.dygraph.rnn`` cells (reference: python/paddle/fluid/dygraph/rnn.py): cuDNN-layout
weights by default (gates i, f, g, o for LSTM; r, z, n for GRU), or the basic layout of
fluid.layers.rnn when ``use_cudnn_impl=False``."""
from __future__ import annotations

import torch

from ...nn.layer.layers import Layer
from ..layers._common import T, W
from ..layers import rnn as LR

__all__ = ["LSTMCell", "GRUCell"]


class LSTMCell(Layer):
    def __init__(self, hidden_size, input_size, param_attr=None, bias_attr=None, gate_activation=None,
                 activation=None, forget_bias=1.0, use_cudnn_impl=True, dtype="float64"):
        super().__init__()
        self._H, self._cudnn, self._fb = hidden_size, use_cudnn_impl, forget_bias
        self._gact, self._act = LR._act(gate_activation or "sigmoid"), LR._act(activation or "tanh")
        H = hidden_size
        if use_cudnn_impl:
            self._weight_ih = self.create_parameter([4 * H, input_size], param_attr, dtype)
            self._weight_hh = self.create_parameter([4 * H, H], param_attr, dtype)
            self._bias_ih = self.create_parameter([4 * H], bias_attr, dtype, is_bias=True)
            self._bias_hh = self.create_parameter([4 * H], bias_attr, dtype, is_bias=True)
        else:
            self._weight = self.create_parameter([input_size + H, 4 * H], param_attr, dtype)
            self._bias = self.create_parameter([4 * H], bias_attr, dtype, is_bias=True)

    def forward(self, input, pre_hidden, pre_cell):
        x, h, c = T(input), T(pre_hidden), T(pre_cell)
        if self._cudnn:
            g = x @ T(self._weight_ih).t() + T(self._bias_ih) + h @ T(self._weight_hh).t() + T(self._bias_hh)
            i, f, gg, o = g.chunk(4, -1)
            c2 = self._gact(f) * c + self._gact(i) * self._act(gg)
            h2 = self._gact(o) * self._act(c2)
        else:
            g = torch.cat([x, h], -1) @ T(self._weight) + T(self._bias)
            i, j, f, o = g.chunk(4, -1)
            c2 = c * self._gact(f + self._fb) + self._gact(i) * self._act(j)
            h2 = self._act(c2) * self._gact(o)
        return W(h2), W(c2)


class GRUCell(Layer):
    def __init__(self, hidden_size, input_size, param_attr=None, bias_attr=None, gate_activation=None,
                 activation=None, use_cudnn_impl=True, dtype="float64"):
        super().__init__()
        self._H, self._cudnn = hidden_size, use_cudnn_impl
        self._gact, self._act = LR._act(gate_activation or "sigmoid"), LR._act(activation or "tanh")
        H = hidden_size
        if use_cudnn_impl:
            self._weight_ih = self.create_parameter([3 * H, input_size], param_attr, dtype)
            self._weight_hh = self.create_parameter([3 * H, H], param_attr, dtype)
            self._bias_ih = self.create_parameter([3 * H], bias_attr, dtype, is_bias=True)
            self._bias_hh = self.create_parameter([3 * H], bias_attr, dtype, is_bias=True)
        else:
            self._gate_weight = self.create_parameter([input_size + H, 2 * H], param_attr, dtype)
            self._gate_bias = self.create_parameter([2 * H], bias_attr, dtype, is_bias=True)
            self._candidate_weight = self.create_parameter([input_size + H, H], param_attr, dtype)
            self._candidate_bias = self.create_parameter([H], bias_attr, dtype, is_bias=True)

    def forward(self, input, pre_hidden):
        x, h = T(input), T(pre_hidden)
        if self._cudnn:
            gi = x @ T(self._weight_ih).t() + T(self._bias_ih)
            gh = h @ T(self._weight_hh).t() + T(self._bias_hh)
            ir, iz, inn = gi.chunk(3, -1)
            hr, hz, hn = gh.chunk(3, -1)
            r, z = self._gact(ir + hr), self._gact(iz + hz)
            n = self._act(inn + r * hn)
            return W((1 - z) * n + z * h)
        g = self._gact(torch.cat([x, h], -1) @ T(self._gate_weight) + T(self._gate_bias))
        r, u = g.chunk(2, -1)
        c = self._act(torch.cat([x, r * h], -1) @ T(self._candidate_weight) + T(self._candidate_bias))
        return W(u * h + (1 - u) * c)
