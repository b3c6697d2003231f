"""Recurrent layers (reference: python/paddle/nn/layer/rnn.py).

Cells keep Paddle's parameter names/shapes (``weight_ih`` [gates*H, in] …), and
the multi-layer SimpleRNN/LSTM/GRU keep Paddle's sublayer structure
(``0.cell`` / ``0.cell_fw`` …) so state dicts round-trip. Full-sequence layers
run each (layer, direction) as one fused recurrent kernel call (PyTorch-ROCm
``_VF`` RNN over the same parameters) instead of a Python time loop.
"""
from __future__ import annotations

import math

import torch

from ...framework.core import Tensor, _wrap
from .. import functional as F
from .. import initializer as I
from .container import LayerList
from .layers import Layer

__all__ = ["RNNCellBase", "SimpleRNNCell", "LSTMCell", "GRUCell", "RNN", "BiRNN", "SimpleRNN", "LSTM", "GRU"]


class RNNCellBase(Layer):
    def get_initial_states(self, batch_ref, shape=None, dtype=None, init_value=0.0, batch_dim_idx=0):
        b = batch_ref._t.shape[batch_dim_idx] if isinstance(batch_ref, Tensor) else batch_ref
        shp = self.state_shape
        dt = self.weight_ih._t.dtype
        dev = self.weight_ih._t.device
        if isinstance(shp[0], (list, tuple)):
            return tuple(_wrap(torch.full([b] + list(s), init_value, dtype=dt, device=dev)) for s in shp)
        return _wrap(torch.full([b] + list(shp), init_value, dtype=dt, device=dev))


class _CellMixin:
    _gates = 1
    _mode = "RNN_TANH"

    def _build(self, input_size, hidden_size, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr):
        self.input_size, self.hidden_size = input_size, hidden_size
        std = 1.0 / math.sqrt(hidden_size)
        g = self._gates
        self.weight_ih = self.create_parameter([g * hidden_size, input_size], weight_ih_attr, default_initializer=I.Uniform(-std, std))
        self.weight_hh = self.create_parameter([g * hidden_size, hidden_size], weight_hh_attr, default_initializer=I.Uniform(-std, std))
        self.bias_ih = self.create_parameter([g * hidden_size], bias_ih_attr, is_bias=True, default_initializer=I.Uniform(-std, std))
        self.bias_hh = self.create_parameter([g * hidden_size], bias_hh_attr, is_bias=True, default_initializer=I.Uniform(-std, std))

    def _flat(self):
        ws = [self.weight_ih._t, self.weight_hh._t]
        if self.bias_ih is not None:
            ws += [self.bias_ih._t, self.bias_hh._t]
        return ws


class SimpleRNNCell(_CellMixin, RNNCellBase):
    _gates = 1

    def __init__(self, input_size, hidden_size, activation="tanh", weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__()
        self.activation = activation
        self._mode = "RNN_TANH" if activation == "tanh" else "RNN_RELU"
        self._build(input_size, hidden_size, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)

    @property
    def state_shape(self):
        return (self.hidden_size,)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        f = torch.rnn_tanh_cell if self.activation == "tanh" else torch.rnn_relu_cell
        h = f(inputs._t, states._t, self.weight_ih._t, self.weight_hh._t,
              None if self.bias_ih is None else self.bias_ih._t, None if self.bias_hh is None else self.bias_hh._t)
        return _wrap(h), _wrap(h)


class LSTMCell(_CellMixin, RNNCellBase):
    _gates = 4
    _mode = "LSTM"

    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, name=None):
        super().__init__()
        self._build(input_size, hidden_size, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)

    @property
    def state_shape(self):
        return ((self.hidden_size,), (self.hidden_size,))

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        h, c = torch.lstm_cell(inputs._t, (states[0]._t, states[1]._t), self.weight_ih._t, self.weight_hh._t,
                               None if self.bias_ih is None else self.bias_ih._t, None if self.bias_hh is None else self.bias_hh._t)
        return _wrap(h), (_wrap(h), _wrap(c))


class GRUCell(_CellMixin, RNNCellBase):
    _gates = 3
    _mode = "GRU"

    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, name=None):
        super().__init__()
        self._build(input_size, hidden_size, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)

    @property
    def state_shape(self):
        return (self.hidden_size,)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        h = torch.gru_cell(inputs._t, states._t, self.weight_ih._t, self.weight_hh._t,
                           None if self.bias_ih is None else self.bias_ih._t, None if self.bias_hh is None else self.bias_hh._t)
        return _wrap(h), _wrap(h)


def _run_seq(cell, x, init, reverse, seq_len=None):
    """Run one direction of one layer over x [B, T, in] (batch-first) with the fused recurrent kernel."""
    if reverse:
        x = x.flip(1)
    ws = cell._flat()
    has_b = cell.bias_ih is not None
    if cell._mode == "LSTM":
        h0, c0 = init
        out, h, c = torch._VF.lstm(x, (h0.unsqueeze(0), c0.unsqueeze(0)), ws, has_b, 1, 0.0, False, False, True)
        state = (h[0], c[0])
    elif cell._mode == "GRU":
        out, h = torch._VF.gru(x, init.unsqueeze(0), ws, has_b, 1, 0.0, False, False, True)
        state = h[0]
    else:
        f = torch._VF.rnn_tanh if cell._mode == "RNN_TANH" else torch._VF.rnn_relu
        out, h = f(x, init.unsqueeze(0), ws, has_b, 1, 0.0, False, False, True)
        state = h[0]
    if reverse:
        out = out.flip(1)
    return out, state


def _zero_state(cell, x):
    b = x.shape[0]
    z = torch.zeros(b, cell.hidden_size, dtype=x.dtype, device=x.device)
    return (z, z.clone()) if cell._mode == "LSTM" else z


class RNN(Layer):
    def __init__(self, cell, is_reverse=False, time_major=False):
        super().__init__()
        self.cell, self.is_reverse, self.time_major = cell, is_reverse, time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        x = inputs._t
        if self.time_major:
            x = x.transpose(0, 1)
        if isinstance(self.cell, _CellMixin) and sequence_length is None:
            init = _zero_state(self.cell, x) if initial_states is None else (
                tuple(s._t for s in initial_states) if isinstance(initial_states, (list, tuple)) else initial_states._t)
            out, st = _run_seq(self.cell, x, init, self.is_reverse)
            if self.time_major:
                out = out.transpose(0, 1)
            st = tuple(_wrap(s) for s in st) if isinstance(st, tuple) else _wrap(st)
            return _wrap(out), st
        # generic cell: python time loop (supports any user RNNCellBase and masking)
        T = x.shape[1]
        states = initial_states
        outs = []
        steps = range(T - 1, -1, -1) if self.is_reverse else range(T)
        mask = None
        if sequence_length is not None:
            mask = torch.arange(T, device=x.device)[None, :] < sequence_length._t[:, None]
        for t in steps:
            o, new_states = self.cell(_wrap(x[:, t]), states)
            if mask is not None and states is not None:
                m = mask[:, t:t + 1]
                new_states = _mask_states(new_states, states, m)
            states = new_states
            outs.append(o._t)
        if self.is_reverse:
            outs = outs[::-1]
        out = torch.stack(outs, 1)
        if self.time_major:
            out = out.transpose(0, 1)
        return _wrap(out), states


def _mask_states(new, old, m):
    if isinstance(new, (list, tuple)):
        return type(new)(_mask_states(a, b, m) for a, b in zip(new, old))
    return _wrap(torch.where(m.to(torch.bool), new._t, old._t))


class BiRNN(Layer):
    def __init__(self, cell_fw, cell_bw, time_major=False):
        super().__init__()
        self.cell_fw, self.cell_bw, self.time_major = cell_fw, cell_bw, time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        fw = RNN(self.cell_fw, False, self.time_major)
        bw = RNN(self.cell_bw, True, self.time_major)
        s_fw, s_bw = (None, None) if initial_states is None else initial_states
        o1, st1 = fw(inputs, s_fw, sequence_length)
        o2, st2 = bw(inputs, s_bw, sequence_length)
        return _wrap(torch.cat([o1._t, o2._t], -1)), (st1, st2)


class _RNNBase(LayerList):
    _cell_cls = SimpleRNNCell

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, **cell_kw):
        super().__init__()
        bidir = direction in ("bidirect", "bidirectional")
        self.num_directions = 2 if bidir else 1
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.time_major, self.dropout = time_major, dropout
        kw = dict(weight_ih_attr=weight_ih_attr, weight_hh_attr=weight_hh_attr, bias_ih_attr=bias_ih_attr,
                  bias_hh_attr=bias_hh_attr, **cell_kw)
        for i in range(num_layers):
            ins = input_size if i == 0 else hidden_size * self.num_directions
            if bidir:
                self.append(BiRNN(self._cell_cls(ins, hidden_size, **kw), self._cell_cls(ins, hidden_size, **kw), time_major))
            else:
                self.append(RNN(self._cell_cls(ins, hidden_size, **kw), False, time_major))
        # the reference also registers every cell parameter on the RNN itself as
        # weight_ih_l{k}[_reverse] / weight_hh_l{k} / bias_ih_l{k} / bias_hh_l{k}, so its state
        # dicts carry both key sets (python/paddle/nn/layer/rnn.py:941-950)
        names = []
        for layer in range(num_layers):
            for d in range(self.num_directions):
                sfx = "_reverse" if d == 1 else ""
                names += [f"weight_ih_l{layer}{sfx}", f"weight_hh_l{layer}{sfx}"]
                if bias_ih_attr is not False:
                    names.append(f"bias_ih_l{layer}{sfx}")
                if bias_hh_attr is not False:
                    names.append(f"bias_hh_l{layer}{sfx}")
        for name, param in zip(names, [p for p in self.parameters() if p is not None]):
            setattr(self, name, param)

    def forward(self, inputs, initial_states=None, sequence_length=None):
        x = inputs
        is_lstm = self._cell_cls is LSTMCell
        finals_h, finals_c = [], []
        init = None
        if initial_states is not None:
            if is_lstm:
                h0, c0 = initial_states[0]._t, initial_states[1]._t
            else:
                h0 = initial_states._t
        for i, layer in enumerate(self):
            if initial_states is not None:
                if self.num_directions == 1:
                    init = (_wrap(h0[i]), _wrap(c0[i])) if is_lstm else _wrap(h0[i])
                else:
                    f = 2 * i
                    init = (((_wrap(h0[f]), _wrap(c0[f])), (_wrap(h0[f + 1]), _wrap(c0[f + 1]))) if is_lstm
                            else (_wrap(h0[f]), _wrap(h0[f + 1])))
            x, st = layer(x, init, sequence_length)
            if self.dropout and self.training and i < len(self) - 1:
                x = F.dropout(x, self.dropout, training=True)
            sts = st if self.num_directions == 2 else (st,)
            for s in sts:
                if is_lstm:
                    finals_h.append(s[0]._t)
                    finals_c.append(s[1]._t)
                else:
                    finals_h.append(s._t)
        h = _wrap(torch.stack(finals_h, 0))
        if is_lstm:
            return x, (h, _wrap(torch.stack(finals_c, 0)))
        return x, h


class SimpleRNN(_RNNBase):
    _cell_cls = SimpleRNNCell

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 activation="tanh", weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__(input_size, hidden_size, num_layers, direction, time_major, dropout, weight_ih_attr,
                         weight_hh_attr, bias_ih_attr, bias_hh_attr, activation=activation)


class LSTM(_RNNBase):
    _cell_cls = LSTMCell

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__(input_size, hidden_size, num_layers, direction, time_major, dropout, weight_ih_attr,
                         weight_hh_attr, bias_ih_attr, bias_hh_attr)


class GRU(_RNNBase):
    _cell_cls = GRUCell

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__(input_size, hidden_size, num_layers, direction, time_major, dropout, weight_ih_attr,
                         weight_hh_attr, bias_ih_attr, bias_hh_attr)
