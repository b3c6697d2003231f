"""Recurrent layers (reference: python/paddle/nn/layer/rnn.py).

Cells keep Paddle's parameter names/shapes (``weight_ih`` [gates*H, in] …), and
the multi-layer SimpleRNN/LSTM/GRU keep Paddle's sublayer structure
(``0.cell`` / ``0.cell_fw`` …) so state dicts round-trip. Full-sequence layers
(``SimpleRNN / LSTM / GRU`` and ``RNN(cell)`` over a plain cell) run as ONE reference ``rnn`` op
(nn/functional/rnn_op.py): on the GPU the own HIP recurrent kernels (csrc/kernels/rnn.hip), on
the CPU torch's recurrent kernels; in a static Program it records as one op (reference
rnn.py:1008-1056 ``_cudnn_impl``) and saves as the reference ``rnn`` op type. User cells run a
time loop over the cell, whose composite form records op by op.
"""
from __future__ import annotations

import math

import torch

from ...framework import core as _core
from ...framework.core import Tensor, _wrap
from .. import functional as F
from .. import initializer as I
from .container import LayerList
from .layers import Layer

__all__ = ["RNNCellBase", "SimpleRNNCell", "LSTMCell", "GRUCell", "RNN", "BiRNN", "SimpleRNN", "LSTM", "GRU"]


class RNNCellBase(Layer):
    def get_initial_states(self, batch_ref, shape=None, dtype=None, init_value=0.0, batch_dim_idx=0):
        shp = self.state_shape
        dt = self.weight_ih._t.dtype
        dev = self.weight_ih._t.device
        if _core._mode.static and isinstance(batch_ref, Tensor):   # the -1 batch: a recorded op
            from ..functional.rnn_op import batch_full
            if isinstance(shp[0], (list, tuple)):
                return tuple(batch_full(batch_ref, list(s), init_value, batch_dim_idx, dt) for s in shp)
            return batch_full(batch_ref, list(shp), init_value, batch_dim_idx, dt)
        b = batch_ref._t.shape[batch_dim_idx] if isinstance(batch_ref, Tensor) else batch_ref
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

    def _gate_preacts(self, inputs, h):
        """x W_ih^T + b_ih and h W_hh^T + b_hh as registered ops (recordable, own GEMMs on GPU)"""
        from ...tensor import matmul
        gi = matmul(inputs, self.weight_ih, transpose_y=True)
        gh = matmul(h, self.weight_hh, transpose_y=True)
        if self.bias_ih is not None:
            gi = gi + self.bias_ih
        if self.bias_hh is not None:
            gh = gh + self.bias_hh
        return gi, gh

    def _composite_ok(self, inputs):
        return _core._mode.static or inputs._t.is_cuda

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
        if self._composite_ok(inputs):
            gi, gh = self._gate_preacts(inputs, states)
            h = F.tanh(gi + gh) if self.activation == "tanh" else F.relu(gi + gh)
            return h, h
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
        if self._composite_ok(inputs):
            from ...tensor import split
            gi, gh = self._gate_preacts(inputs, states[0])
            i, f, g, o = split(gi + gh, 4, axis=-1)
            c = F.sigmoid(f) * states[1] + F.sigmoid(i) * F.tanh(g)
            h = F.sigmoid(o) * F.tanh(c)
            return h, (h, c)
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
        if self._composite_ok(inputs):
            from ...tensor import split
            gi, gh = self._gate_preacts(inputs, states)
            xr, xz, xc = split(gi, 3, axis=-1)
            hr, hz, hc = split(gh, 3, axis=-1)
            r = F.sigmoid(xr + hr)
            z = F.sigmoid(xz + hz)
            c = F.tanh(xc + r * hc)
            h = (states - c) * z + c
            return h, h
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
        ws = _cell_weights(self.cell)
        if ws is not None and (sequence_length is None or not self.is_reverse):
            return self._op_forward(inputs, initial_states, sequence_length, ws)
        if _core._mode.static or inputs._t.is_cuda:
            # recorded step by step through the cells' composite form (static); on the GPU the
            # cells' registered ops (own GEMMs) instead of torch's fused recurrent kernels
            return self._loop_forward(inputs, initial_states, sequence_length)
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


    def _op_forward(self, inputs, initial_states, sequence_length, ws):
        """the cell over the sequence as ONE single-layer rnn op (a reverse pass runs on the
        time-flipped sequence)"""
        from ..functional import rnn_op as R
        from ...tensor import transpose, flip, unsqueeze, squeeze
        cell = self.cell
        mode = _cell_mode(cell)
        ncomp = 2 if mode == "LSTM" else 1
        batch_index = 1 if self.time_major else 0
        if initial_states is None:
            states = []
            for _ in range(ncomp):
                st = R.init_state(inputs, 1, cell.hidden_size, batch_index)
                R.mark_init_state(st, inputs, 1, cell.hidden_size, batch_index)
                states.append(st)
        else:
            sts = list(initial_states) if isinstance(initial_states, (list, tuple)) else [initial_states]
            states = [unsqueeze(s_, 0) for s_ in sts]
        x = inputs if self.time_major else transpose(inputs, [1, 0, 2])
        if self.is_reverse:
            x = flip(x, [0])
        attrs = {"dropout_prob": 0.0, "is_bidirec": False, "input_size": int(cell.input_size),
                 "hidden_size": int(cell.hidden_size), "num_layers": 1, "mode": mode, "is_test": not self.training}
        out, state = R.rnn_op(x, states, ws, sequence_length, **attrs)
        R.mark_reference_form(out, state, x, states, ws, sequence_length, attrs)
        if self.is_reverse:
            out = flip(out, [0])
        if not self.time_major:
            out = transpose(out, [1, 0, 2])
        state = [squeeze(s_, [0]) for s_ in state]
        return out, (tuple(state) if ncomp == 2 else state[0])

    def _loop_forward(self, inputs, initial_states, sequence_length):
        """time loop over the cell with registered ops only (static recording)"""
        from ...tensor import transpose, stack, where, unsqueeze
        x = inputs if self.time_major else transpose(inputs, [1, 0, 2])
        T = x.shape[0]
        states = initial_states
        outs = [None] * T
        for t in (range(T - 1, -1, -1) if self.is_reverse else range(T)):
            o, new_states = self.cell(x[t], states)
            if sequence_length is not None and states is not None:
                m = unsqueeze(sequence_length > t, 1)
                new_states = _mask_states_op(new_states, states, m, where)
                o = where(m, o, o * 0)
            states = new_states
            outs[t] = o
        out = stack(outs, 0)
        if not self.time_major:
            out = transpose(out, [1, 0, 2])
        return out, states


def _cell_mode(cell):
    if isinstance(cell, LSTMCell):
        return "LSTM"
    if isinstance(cell, GRUCell):
        return "GRU"
    return "RNN_RELU" if getattr(cell, "activation", "tanh") == "relu" else "RNN_TANH"


def _cell_weights(cell):
    """a plain cell's parameters as the rnn op's weight list (None for user cells or mixed biases)"""
    if type(cell) not in (SimpleRNNCell, LSTMCell, GRUCell):
        return None
    hb = (cell.bias_ih is not None, cell.bias_hh is not None)
    if hb == (True, True):
        return [cell.weight_ih, cell.weight_hh, cell.bias_ih, cell.bias_hh]
    if hb == (False, False):
        return [cell.weight_ih, cell.weight_hh]
    return None


def _mask_states_op(new, old, m, where):
    if isinstance(new, (list, tuple)):
        return type(new)(_mask_states_op(a, b, m, where) for a, b in zip(new, old))
    return where(m, new, old)


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

    _MODE = "RNN_TANH"

    def _op_mode(self):
        if self._cell_cls is LSTMCell:
            return "LSTM"
        if self._cell_cls is GRUCell:
            return "GRU"
        return "RNN_RELU" if getattr(self[0].cell if self.num_directions == 1 else self[0].cell_fw,
                                      "activation", "tanh") == "relu" else "RNN_TANH"

    def _cells(self):
        out = []
        for layer in self:
            out += [layer.cell] if self.num_directions == 1 else [layer.cell_fw, layer.cell_bw]
        return out

    @property
    def _all_weights(self):
        """the reference op's WeightList (RNNBase.flatten_parameters, rnn.py:953-962): every cell's
        weight_ih, weight_hh, then every cell's bias_ih, bias_hh; None when the cells are not all
        plain cells with the same bias layout (then the per-cell path runs, as the reference's
        could_use_cudnn = False)"""
        cells = self._cells()
        if not all(type(c) is self._cell_cls for c in cells):
            return None
        nb = {(c.bias_ih is not None, c.bias_hh is not None) for c in cells}
        if len(nb) != 1 or nb.pop() not in ((True, True), (False, False)):
            return None
        ws = [w for c in cells for w in (c.weight_ih, c.weight_hh)]
        if cells[0].bias_ih is not None:
            ws += [b for c in cells for b in (c.bias_ih, c.bias_hh)]
        return ws

    def forward(self, inputs, initial_states=None, sequence_length=None):
        ws = self._all_weights
        if ws is not None:
            return self._op_forward(inputs, initial_states, sequence_length, ws)
        return self._cell_forward(inputs, initial_states, sequence_length)

    def _op_forward(self, inputs, initial_states, sequence_length, ws):
        """ONE rnn op over all layers and directions (reference _cudnn_impl): HIP recurrent
        kernels on the GPU, one recorded op in a static Program"""
        from ..functional import rnn_op as R
        from ...tensor import transpose
        mode = self._op_mode()
        ncomp = 2 if mode == "LSTM" else 1
        batch_index = 1 if self.time_major else 0
        n = self.num_layers * self.num_directions
        if initial_states is None:
            states = []
            for _ in range(ncomp):
                st = R.init_state(inputs, n, self.hidden_size, batch_index)
                R.mark_init_state(st, inputs, n, self.hidden_size, batch_index)
                states.append(st)
        else:
            states = list(initial_states) if isinstance(initial_states, (list, tuple)) else [initial_states]
        x = inputs if self.time_major else transpose(inputs, [1, 0, 2])
        attrs = {"dropout_prob": float(self.dropout), "is_bidirec": self.num_directions == 2,
                 "input_size": int(self.input_size), "hidden_size": int(self.hidden_size),
                 "num_layers": int(self.num_layers), "mode": mode, "is_test": not self.training}
        out, state = R.rnn_op(x, states, ws, sequence_length, **attrs)
        R.mark_reference_form(out, state, x, states, ws, sequence_length, attrs)
        if not self.time_major:
            out = transpose(out, [1, 0, 2])
        return out, (tuple(state) if ncomp == 2 else state[0])

    def _cell_forward(self, inputs, initial_states=None, sequence_length=None):
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
