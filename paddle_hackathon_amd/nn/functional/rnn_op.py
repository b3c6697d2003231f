"""The ``rnn`` operator as one recordable op (reference: python/paddle/nn/layer/rnn.py:1008-1056
``RNNBase._cudnn_impl`` -> ``append_op(type="rnn")``; paddle/fluid/operators/rnn_op.cc).

``rnn_op`` takes the reference op's inputs and attributes — Input [T, B, I] (time-major),
PreState [h0] / [h0, c0] ([L*D, B, H]), WeightList (every (layer, direction)'s weight_ih, weight_hh,
then every bias_ih, bias_hh), SequenceLength [B] — and returns (Out [T, B, D*H], State). It is a
registered op, so in a static Program (program_guard, ``to_static``, ``jit.save``) it records as
ONE op whose shapes come from a pure-shape InferMeta; ``nn.SimpleRNN / LSTM / GRU`` mark it with
the reference form (``rnn`` with Reserve / DropoutState outputs) so saved programs carry the
reference op type, and static/ref_ops.py converts a reference ``rnn`` op back to it. Kernels:
ops/rnn.py (HIP time loop on the GPU)."""
from __future__ import annotations

import torch

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops

__all__ = []


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def rnn_op(input, pre_state, weight_list, sequence_length=None, dropout_prob=0.0, is_bidirec=False, input_size=10,
           hidden_size=100, num_layers=1, mode="LSTM", is_test=False):
    from ...ops import rnn as _rnn
    pre = [_t(s) for s in (pre_state if isinstance(pre_state, (list, tuple)) else [pre_state])]
    ws = [_t(w) for w in weight_list]
    sl = None if sequence_length is None else _t(sequence_length)
    out, state = _rnn.rnn(_t(input), pre, ws, sl, float(dropout_prob), bool(is_bidirec), int(input_size),
                          int(hidden_size), int(num_layers), str(mode), bool(is_test))
    return _wrap(out), [_wrap(s) for s in state]


def init_state(input, num, hidden_size, batch_dim=1):
    """zeros [num, B, hidden_size] with B = input.shape[batch_dim] (the reference creates the
    default initial states with fill_constant_batch_size_like)"""
    x = _t(input)
    return _wrap(torch.zeros(int(num), x.shape[batch_dim], int(hidden_size), dtype=x.dtype, device=x.device))


def batch_full(input, shape, value=0.0, batch_dim=0, dtype=None):
    """full([B] + shape, value) with B = input.shape[batch_dim] (a cell's initial state in a static
    Program, where B is the -1 batch)"""
    x = _t(input)
    return _wrap(torch.full([x.shape[batch_dim]] + [int(d) for d in shape], float(value),
                            dtype=dtype or x.dtype, device=x.device))


register_ops(globals(), ["rnn_op", "init_state", "batch_full"])


def _meta_rnn(input, pre_state, weight_list, sequence_length=None, dropout_prob=0.0, is_bidirec=False, input_size=10,
              hidden_size=100, num_layers=1, mode="LSTM", is_test=False):
    """pure-shape InferMeta (the reference RnnInferMeta: Out [T, B, D*H], State like PreState)"""
    x = _t(input)
    D = 2 if is_bidirec else 1
    out = _wrap(torch.empty(x.shape[0], x.shape[1], D * int(hidden_size), dtype=x.dtype, device="meta"))
    pre = pre_state if isinstance(pre_state, (list, tuple)) else [pre_state]
    return out, [_wrap(torch.empty(tuple(_t(s).shape), dtype=x.dtype, device="meta")) for s in pre]


def _register_meta():
    from ...static.program import register_infer_meta
    register_infer_meta("rnn_op")(_meta_rnn)


_register_meta()


def mark_reference_form(out, state, input, pre_state, weight_list, sequence_length, attrs):
    """static Programs: the recorded op is written as the reference ``rnn`` op (no-op in dygraph)"""
    from ...framework import core as _core
    if not _core._mode.static or getattr(out, "op", None) is None:
        return
    from ...static.program import set_ref_op
    from ...static.ref_emit import _tmp_var
    reserve = _tmp_var(out.name + "@rnn_reserve", out, [-1], torch.uint8)
    dstate = _tmp_var(out.name + "@rnn_dropout_state", out, [-1], torch.uint8)
    ins = {"Input": [input], "PreState": list(pre_state), "WeightList": list(weight_list)}
    if sequence_length is not None:
        ins["SequenceLength"] = [sequence_length]
    set_ref_op(out, "rnn", ins, {"Out": [out], "State": list(state), "Reserve": [reserve], "DropoutState": [dstate]},
               attrs)


def mark_init_state(state, input, num, hidden_size, batch_dim=1):
    from ...framework import core as _core
    if not _core._mode.static or getattr(state, "op", None) is None:
        return
    from ...static.program import set_ref_op
    from ...static import proto as pb
    set_ref_op(state, "fill_constant_batch_size_like", {"Input": [input]}, {"Out": [state]},
               {"shape": [int(num), -1, int(hidden_size)], "value": 0.0, "dtype": pb.vartype_of(_t(input).dtype),
                "input_dim_idx": int(batch_dim), "output_dim_idx": 1, "force_cpu": False})
