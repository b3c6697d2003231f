"""``fluid.contrib.BasicGRUUnit`` / ``BasicLSTMUnit`` with the 1.x signature (reference:
python/paddle/fluid/contrib/layers/rnn_impl.py:25 BasicGRUUnit, :700 BasicLSTMUnit).

``(name_scope, hidden_size, param_attr, bias_attr, gate_activation, activation, dtype)``; the
weights are created on the first call, when the input width is known (the reference's
``_build_once``). Both units run the gates as ONE GEMM over ``[x, h]`` (the fused-gate layout of
the reference: GRU gate weight [in + hidden, 2 * hidden] -> (r, u), candidate weight
[in + hidden, hidden]; LSTM weight [in + hidden, 4 * hidden] -> (i, j, f, o), forget_bias added
to f)."""
from __future__ import annotations

import copy

from ... import tensor as T
from ...nn import functional as F
from ...nn.layer.layers import Layer

__all__ = ["BasicGRUUnit", "BasicLSTMUnit"]


def _suffixed(attr, suffix):
    if attr is not None and getattr(attr, "name", None) is not None:
        a = copy.deepcopy(attr)
        a.name += suffix
        return a
    return attr


class BasicGRUUnit(Layer):
    """h' = u * h + (1 - u) * act(W_c [x, r * h] + b_c),  (r, u) = gate_act(W_g [x, h] + b_g)"""

    def __init__(self, name_scope, hidden_size, param_attr=None, bias_attr=None, gate_activation=None,
                 activation=None, dtype="float32"):
        super().__init__(name_scope=name_scope, dtype=dtype)
        self._hidden_size = int(hidden_size)
        self._param_attr, self._bias_attr = param_attr, bias_attr
        self._gate_activation = gate_activation or F.sigmoid
        self._activation = activation or T.tanh
        self._dtype = dtype
        self._built = False

    def _build_once(self, input, pre_hidden):
        n_in, H = int(input.shape[-1]), self._hidden_size
        assert n_in > 0
        self._gate_weight = self.create_parameter([n_in + H, 2 * H], _suffixed(self._param_attr, "_gate"),
                                                  self._dtype)
        self._candidate_weight = self.create_parameter([n_in + H, H], _suffixed(self._param_attr, "_candidate"),
                                                       self._dtype)
        self._gate_bias = self.create_parameter([2 * H], _suffixed(self._bias_attr, "_gate"), self._dtype,
                                                is_bias=True)
        self._candidate_bias = self.create_parameter([H], _suffixed(self._bias_attr, "_candidate"), self._dtype,
                                                     is_bias=True)
        self._built = True

    def forward(self, input, pre_hidden):
        if not self._built:
            self._build_once(input, pre_hidden)
        g = self._gate_activation(T.matmul(T.concat([input, pre_hidden], 1), self._gate_weight) + self._gate_bias)
        r, u = T.split(g, 2, axis=1)
        c = self._activation(T.matmul(T.concat([input, r * pre_hidden], 1), self._candidate_weight)
                             + self._candidate_bias)
        return u * pre_hidden + (1 - u) * c


class BasicLSTMUnit(Layer):
    """(i, j, f, o) = W [x, h] + b;  c' = c * sig(f + forget_bias) + sig(i) * act(j);
    h' = act(c') * sig(o)"""

    def __init__(self, name_scope, hidden_size, param_attr=None, bias_attr=None, gate_activation=None,
                 activation=None, forget_bias=1.0, dtype="float32"):
        super().__init__(name_scope=name_scope, dtype=dtype)
        self._hidden_size = int(hidden_size)
        self._param_attr, self._bias_attr = param_attr, bias_attr
        self._gate_activation = gate_activation or F.sigmoid
        self._activation = activation or T.tanh
        self._forget_bias = float(forget_bias)
        self._dtype = dtype
        self._built = False

    def _build_once(self, input, pre_hidden, pre_cell):
        n_in, H = int(input.shape[-1]), self._hidden_size
        assert n_in > 0
        self._weight = self.create_parameter([n_in + H, 4 * H], self._param_attr, self._dtype)
        self._bias = self.create_parameter([4 * H], self._bias_attr, self._dtype, is_bias=True)
        self._built = True

    def forward(self, input, pre_hidden, pre_cell):
        if not self._built:
            self._build_once(input, pre_hidden, pre_cell)
        gates = T.matmul(T.concat([input, pre_hidden], 1), self._weight) + self._bias
        i, j, f, o = T.split(gates, 4, axis=-1)
        sg = self._gate_activation
        new_cell = pre_cell * sg(f + self._forget_bias) + sg(i) * self._activation(j)
        new_hidden = self._activation(new_cell) * sg(o)
        return new_hidden, new_cell
