"""``fluid.layers`` recurrent layers and decoding (reference: python/paddle/fluid/layers/rnn.py;
ops paddle/fluid/operators/{lstm,lstmp,gru,gru_unit,lstm_unit,beam_search,
beam_search_decode}_op.h).

The fluid cells build their weights on first call (input size inferred), with the 1.x gate
layouts: ``LSTMCell`` gates = [x, h] W + b split as (i, j, f, o) with ``forget_bias``;
``GRUCell`` gates (r, u) then candidate on [x, r * h]. ``dynamic_lstm`` / ``dynamic_gru`` take
LoD inputs already projected to 4H / 3H and run per sequence (gate order candidate, input,
forget, output for LSTM; update, reset | candidate for GRU).
"""
from __future__ import annotations

import torch

from ...framework.core import Tensor
from ...framework.dispatch import static_op
from ...nn.layer.layers import Layer
from ._common import fparam as _create_parameter
from ...nn import decode as _decode
from ...nn.layer.rnn import LSTM as _LSTM
from ._common import T, W, dev, to_padded, from_padded
from .. import core as fcore

__all__ = ["RNNCell", "GRUCell", "LSTMCell", "Decoder", "BeamSearchDecoder", "rnn", "birnn", "dynamic_decode",
           "DecodeHelper", "TrainingHelper", "GreedyEmbeddingHelper", "SampleEmbeddingHelper", "BasicDecoder",
           "dynamic_lstm", "dynamic_lstmp", "dynamic_gru", "gru_unit", "lstm_unit", "lstm", "beam_search",
           "beam_search_decode"]

_ACT = {"sigmoid": torch.sigmoid, "tanh": torch.tanh, "relu": torch.relu, "identity": lambda x: x,
        None: lambda x: x}


def _act(a):
    return a if callable(a) else _ACT[a]


class RNNCell(Layer):
    """base of the fluid cells: ``call(inputs, states) -> (outputs, new_states)``"""

    def get_initial_states(self, batch_ref, shape=None, dtype="float32", init_value=0.0, batch_dim_idx=0):
        b = T(batch_ref).shape[batch_dim_idx]
        shp = shape if shape is not None else self.state_shape

        def mk(s):
            if isinstance(s, (list, tuple)) and s and isinstance(s[0], (list, tuple)):
                return [mk(x) for x in s]
            return W(torch.full([b] + list(s), init_value, dtype=fcore.convert_dtype(dtype), device=dev()))
        return mk(shp)

    @property
    def state_shape(self):
        raise NotImplementedError

    def forward(self, inputs, states, **kwargs):
        return self.call(inputs, states, **kwargs)


class LSTMCell(RNNCell):
    def __init__(self, hidden_size, param_attr=None, bias_attr=None, gate_activation=None, activation=None,
                 forget_bias=1.0, dtype="float32", name="LSTMCell"):
        super().__init__()
        self.hidden_size, self.param_attr, self.bias_attr = hidden_size, param_attr, bias_attr
        self.gate_act, self.act = _act(gate_activation or "sigmoid"), _act(activation or "tanh")
        self.forget_bias, self.dtype = forget_bias, dtype
        self.weight = None

    @property
    def state_shape(self):
        return [[self.hidden_size], [self.hidden_size]]

    def _build(self, in_size):
        self.weight = self.create_parameter([in_size + self.hidden_size, 4 * self.hidden_size], self.param_attr)
        self.bias = self.create_parameter([4 * self.hidden_size], self.bias_attr, is_bias=True)

    def call(self, inputs, states):
        x = T(inputs)
        h, c = T(states[0]), T(states[1])
        if self.weight is None:
            self._build(x.shape[-1])
        g = torch.cat([x, h], -1) @ T(self.weight) + T(self.bias)
        i, j, f, o = g.chunk(4, -1)
        c2 = c * self.gate_act(f + self.forget_bias) + self.gate_act(i) * self.act(j)
        h2 = self.act(c2) * self.gate_act(o)
        return W(h2), [W(h2), W(c2)]


class GRUCell(RNNCell):
    def __init__(self, hidden_size, param_attr=None, bias_attr=None, gate_activation=None, activation=None,
                 dtype="float32", name="GRUCell"):
        super().__init__()
        self.hidden_size, self.param_attr, self.bias_attr = hidden_size, param_attr, bias_attr
        self.gate_act, self.act = _act(gate_activation or "sigmoid"), _act(activation or "tanh")
        self.dtype = dtype
        self.gate_w = None

    @property
    def state_shape(self):
        return [self.hidden_size]

    def _build(self, in_size):
        H = self.hidden_size
        self.gate_w = self.create_parameter([in_size + H, 2 * H], self.param_attr)
        self.gate_b = self.create_parameter([2 * H], self.bias_attr, is_bias=True)
        self.cand_w = self.create_parameter([in_size + H, H], self.param_attr)
        self.cand_b = self.create_parameter([H], self.bias_attr, is_bias=True)

    def call(self, inputs, states):
        x, h = T(inputs), T(states)
        if self.gate_w is None:
            self._build(x.shape[-1])
        g = self.gate_act(torch.cat([x, h], -1) @ T(self.gate_w) + T(self.gate_b))
        r, u = g.chunk(2, -1)
        c = self.act(torch.cat([x, r * h], -1) @ T(self.cand_w) + T(self.cand_b))
        h2 = u * h + (1 - u) * c
        return W(h2), W(h2)


def _map(fn, s):
    if isinstance(s, (list, tuple)):
        return type(s)(_map(fn, x) for x in s)
    return fn(s)


def rnn(cell, inputs, initial_states=None, sequence_length=None, time_major=False, is_reverse=False, **kwargs):
    """unrolled recurrence of ``cell`` over ``inputs`` [B, T, ...] (or [T, B, ...]); steps past a
    sequence's length keep its state and output zeros -> (outputs, final_states)"""
    x = T(inputs)
    if not time_major:
        x = x.transpose(0, 1)
    steps, B = x.shape[0], x.shape[1]
    states = initial_states if initial_states is not None else cell.get_initial_states(W(x[0]))
    lens = T(sequence_length).reshape(-1).long() if sequence_length is not None else None
    order = range(steps - 1, -1, -1) if is_reverse else range(steps)
    outs = [None] * steps
    for t in order:
        o, new = cell(W(x[t]), states, **kwargs)
        if lens is not None:
            m = (t < lens).to(T(o).dtype).reshape(B, *([1] * (T(o).dim() - 1)))
            o = W(T(o) * m)
            new = _map(lambda pair: pair, new)
            flat_new, flat_old = _flatten(new), _flatten(states)
            merged = [W(T(a) * m + T(b) * (1 - m)) for a, b in zip(flat_new, flat_old)]
            new = _unflatten(new, merged)
        outs[t] = T(o)
        states = new
    y = torch.stack(outs, 0)
    if not time_major:
        y = y.transpose(0, 1)
    return W(y), states


def _flatten(s):
    if isinstance(s, (list, tuple)):
        return [v for x in s for v in _flatten(x)]
    return [s]


def _unflatten(like, vals):
    it = iter(vals)

    def build(s):
        if isinstance(s, (list, tuple)):
            return type(s)(build(x) for x in s)
        return next(it)
    return build(like)


def birnn(cell_fw, cell_bw, inputs, initial_states=None, sequence_length=None, time_major=False, **kwargs):
    s_fw, s_bw = initial_states if initial_states is not None else (None, None)
    o_fw, f_fw = rnn(cell_fw, inputs, s_fw, sequence_length, time_major, False, **kwargs)
    o_bw, f_bw = rnn(cell_bw, inputs, s_bw, sequence_length, time_major, True, **kwargs)
    return W(torch.cat([T(o_fw), T(o_bw)], -1)), (f_fw, f_bw)


Decoder = _decode.Decoder
BeamSearchDecoder = _decode.BeamSearchDecoder


def dynamic_decode(decoder, inits=None, max_step_num=None, output_time_major=False, impute_finished=False,
                   is_test=False, return_length=False, **kwargs):
    if isinstance(decoder, BasicDecoder):
        return decoder._decode(inits, max_step_num, output_time_major, return_length, **kwargs)
    return _decode.dynamic_decode(decoder, inits, max_step_num, output_time_major, impute_finished, is_test,
                                  return_length, **kwargs)


class DecodeHelper:
    """how a BasicDecoder obtains each step's input and decides when a sequence ends"""

    def initialize(self):
        raise NotImplementedError

    def sample(self, time, outputs, states):
        raise NotImplementedError

    def next_inputs(self, time, outputs, states, sample_ids):
        raise NotImplementedError


class TrainingHelper(DecodeHelper):
    """teacher forcing: step t reads inputs[:, t]; a sequence finishes at its length"""

    def __init__(self, inputs, sequence_length, time_major=False):
        self.inputs = _map(lambda x: T(x) if time_major else T(x).transpose(0, 1), inputs)
        self.lens = T(sequence_length).reshape(-1).long()

    def initialize(self):
        first = _map(lambda x: W(x[0]), self.inputs)
        return first, self.lens == 0

    def sample(self, time, outputs, states):
        return W(T(outputs).argmax(-1))

    def next_inputs(self, time, outputs, states, sample_ids):
        nt = time + 1
        finished = nt >= self.lens
        steps = _flatten(self.inputs)[0].shape[0]
        nxt = _map(lambda x: W(x[min(nt, steps - 1)]), self.inputs)
        return finished, nxt, states


class GreedyEmbeddingHelper(DecodeHelper):
    def __init__(self, embedding_fn, start_tokens, end_token):
        self.embedding_fn, self.end_token = embedding_fn, end_token
        self.start = T(start_tokens).long()

    def initialize(self):
        return self.embedding_fn(W(self.start)), torch.zeros(self.start.shape[0], dtype=torch.bool,
                                                             device=self.start.device)

    def sample(self, time, outputs, states):
        return W(T(outputs).argmax(-1))

    def next_inputs(self, time, outputs, states, sample_ids):
        ids = T(sample_ids)
        return ids == self.end_token, self.embedding_fn(W(ids)), states


class SampleEmbeddingHelper(GreedyEmbeddingHelper):
    def __init__(self, embedding_fn, start_tokens, end_token, softmax_temperature=None, seed=None):
        super().__init__(embedding_fn, start_tokens, end_token)
        self.temp = softmax_temperature
        self.gen = None
        if seed is not None:
            self.gen = torch.Generator(device=self.start.device)
            self.gen.manual_seed(int(seed))

    def sample(self, time, outputs, states):
        logits = T(outputs).float()
        if self.temp is not None:
            logits = logits / self.temp
        return W(torch.multinomial(torch.softmax(logits, -1), 1, generator=self.gen).reshape(-1))


class BasicDecoder(_decode.Decoder):
    """cell + helper (+ output_fn): step outputs (cell_outputs, sample_ids)"""

    def __init__(self, cell, helper, output_fn=None):
        self.cell, self.helper, self.output_fn = cell, helper, output_fn

    def initialize(self, initial_cell_states):
        inputs, finished = self.helper.initialize()
        return inputs, initial_cell_states, finished

    def step(self, time, inputs, states, **kwargs):
        out, new = self.cell(inputs, states, **kwargs)
        if self.output_fn is not None:
            out = self.output_fn(out)
        ids = self.helper.sample(time, out, new)
        finished, nxt, new = self.helper.next_inputs(time, out, new, ids)
        return (out, ids), new, nxt, finished

    def _decode(self, inits, max_step_num, time_major, return_length, **kwargs):
        inputs, states, finished = self.initialize(inits)
        outs, ids = [], []
        lens = torch.zeros(finished.shape[0], dtype=torch.long, device=finished.device)
        t = 0
        while True:
            (o, i), states, inputs, fin = self.step(t, inputs, states, **kwargs)
            lens = lens + (~finished).long()
            outs.append(T(o))
            ids.append(T(i))
            finished = finished | fin
            t += 1
            if bool(finished.all()) or (max_step_num is not None and t > max_step_num):
                break
        o, i = torch.stack(outs, 0), torch.stack(ids, 0)
        if not time_major:
            o, i = o.transpose(0, 1), i.transpose(0, 1)
        res = ((W(o), W(i)), states)
        return res + (W(lens),) if return_length else res


# ----------------------------------------------------------------------------- LoD recurrent ops
def _seq_list(x):
    t = T(x)
    off = fcore.lod_of(x)[-1] if fcore.lod_of(x) else [0, t.shape[0]]
    return t, off


def dynamic_lstm(input, size, h_0=None, c_0=None, param_attr=None, bias_attr=None, use_peepholes=True,
                 is_reverse=False, gate_activation="sigmoid", cell_activation="tanh", candidate_activation="tanh",
                 dtype="float32", name=None):
    """``input`` LoD [T, 4H] (already projected); -> (hidden LoD [T, H], cell LoD [T, H])"""
    H = size // 4
    w = _create_parameter([H, 4 * H], dtype, param_attr)
    b = _create_parameter([1, 7 * H if use_peepholes else 4 * H], dtype, bias_attr, is_bias=True)
    out = _lstm_rec(input, H, w, b, None, use_peepholes, is_reverse, gate_activation, cell_activation,
                    candidate_activation, h_0, c_0, None)
    from ...static.program import set_ref_op
    set_ref_op(out, "lstm", {"Input": [input], "Weight": [w], "Bias": [b], "H0": [h_0], "C0": [c_0]},
               {"Hidden": [out[0]], "Cell": [out[1]]},
               {"use_peepholes": bool(use_peepholes), "is_reverse": bool(is_reverse), "gate_activation": gate_activation,
                "cell_activation": cell_activation, "candidate_activation": candidate_activation})
    return out


def _lstm_run(input, H, w, b, proj, peep, reverse, ga, ca, cand, h0, c0, proj_act):
    x, off = _seq_list(input)
    gact, cact, candact = _act(ga), _act(ca), _act(cand)
    wt, bt = T(w), T(b).reshape(-1)
    hs, cs = [None] * x.shape[0], [None] * x.shape[0]
    P = T(proj) if proj is not None else None
    for s in range(len(off) - 1):
        a, e = off[s], off[s + 1]
        rdim = P.shape[1] if P is not None else H
        h = T(h0)[s] if h0 is not None else x.new_zeros(rdim)
        c = T(c0)[s] if c0 is not None else x.new_zeros(H)
        rng = range(e - 1, a - 1, -1) if reverse else range(a, e)
        for t in rng:
            g = x[t] + h @ wt + bt[:4 * H]
            gc, gi, gf, go = g.split(H)
            if peep:
                wic, wfc, woc = bt[4 * H:5 * H], bt[5 * H:6 * H], bt[6 * H:7 * H]
                gi, gf = gi + wic * c, gf + wfc * c
            i, f = gact(gi), gact(gf)
            c = f * c + i * candact(gc)
            if peep:
                go = go + woc * c
            o = gact(go)
            hh = o * cact(c)
            if P is not None:
                hh = _act(proj_act)(hh @ P)
            h = hh
            hs[t], cs[t] = h, c
    lod = fcore.lod_of(input) or [off]
    ho, co = W(torch.stack(hs)), W(torch.stack(cs))
    ho._lod, co._lod = lod, lod
    return ho, co


def dynamic_lstmp(input, size, proj_size, param_attr=None, bias_attr=None, use_peepholes=True, is_reverse=False,
                  gate_activation="sigmoid", cell_activation="tanh", candidate_activation="tanh",
                  proj_activation="tanh", dtype="float32", name=None, h_0=None, c_0=None, cell_clip=None,
                  proj_clip=None):
    """LSTM with a recurrent projection r = proj_act(h W_p) [T, P]; -> (projection, cell)"""
    H = size // 4
    w = _create_parameter([proj_size, 4 * H], dtype, param_attr)
    pw = _create_parameter([H, proj_size], dtype, param_attr)
    b = _create_parameter([1, 7 * H if use_peepholes else 4 * H], dtype, bias_attr, is_bias=True)
    return _lstm_rec(input, H, w, b, pw, use_peepholes, is_reverse, gate_activation, cell_activation,
                     candidate_activation, h_0, c_0, proj_activation)


def _gru_step(x, h, wt, bt, H, gact, cact, origin):
    xu, xr, xc = (x + bt).split(H)
    hu = h @ wt[:, :H]
    hr = h @ wt[:, H:2 * H]
    u, r = gact(xu + hu), gact(xr + hr)
    rh = r * h
    c = cact(xc + rh @ wt[:, 2 * H:])
    hn = u * h + (1 - u) * c if origin else (1 - u) * h + u * c
    return hn, r, rh, c, u


def dynamic_gru(input, size, param_attr=None, bias_attr=None, is_reverse=False, gate_activation="sigmoid",
                candidate_activation="tanh", h_0=None, origin_mode=False):
    """``input`` LoD [T, 3H] (projected); -> hidden LoD [T, H]"""
    H = size
    w = _create_parameter([H, 3 * H], "float32", param_attr)
    b = _create_parameter([1, 3 * H], "float32", bias_attr, is_bias=True)
    out = _gru_rec(input, w, b, H, is_reverse, gate_activation, candidate_activation, h_0, origin_mode)
    from ...static.program import set_ref_op
    set_ref_op(out, "gru", {"Input": [input], "Weight": [w], "Bias": [b], "H0": [h_0]}, {"Hidden": [out]},
               {"activation": candidate_activation, "gate_activation": gate_activation, "is_reverse": bool(is_reverse),
                "origin_mode": bool(origin_mode)})
    return out


def _gru_run(input, w, b, H, is_reverse, gate_activation, candidate_activation, h_0, origin_mode):
    x, off = _seq_list(input)
    wt, bt = T(w), T(b).reshape(-1)
    hs = [None] * x.shape[0]
    for s in range(len(off) - 1):
        a, e = off[s], off[s + 1]
        h = T(h_0)[s] if h_0 is not None else x.new_zeros(H)
        for t in (range(e - 1, a - 1, -1) if is_reverse else range(a, e)):
            h = _gru_step(x[t], h, wt, bt, H, _act(gate_activation), _act(candidate_activation), origin_mode)[0]
            hs[t] = h
    out = W(torch.stack(hs))
    out._lod = fcore.lod_of(input) or [off]
    return out


# the recurrences record ONE op each in a static Program (the parameters are created by the
# builders above; the op type is the reference's lstm / gru)
_lstm_rec = static_op(_lstm_run, "lstm")
_gru_rec = static_op(_gru_run, "gru")


def gru_unit(input, hidden, size, param_attr=None, bias_attr=None, activation="tanh", gate_activation="sigmoid",
             origin_mode=False):
    """one GRU step on [N, 3H] projected input; -> (new hidden, reset_hidden_prev, gate)"""
    H = size // 3
    w = _create_parameter([H, 3 * H], "float32", param_attr)
    b = _create_parameter([1, 3 * H], "float32", bias_attr, is_bias=True)
    return _gru_unit_rec(input, hidden, w, b, H, activation, gate_activation, origin_mode)


def _gru_unit_run(input, hidden, w, b, H, activation, gate_activation, origin_mode):
    x, h = T(input), T(hidden)
    wt, bt = T(w), T(b).reshape(-1)
    xu, xr, xc = (x + bt).split(H, -1)
    u = _act(gate_activation)(xu + h @ wt[:, :H])
    r = _act(gate_activation)(xr + h @ wt[:, H:2 * H])
    rh = r * h
    c = _act(activation)(xc + rh @ wt[:, 2 * H:])
    hn = u * h + (1 - u) * c if origin_mode else (1 - u) * h + u * c
    return W(hn), W(rh), W(torch.cat([u, r, c], -1))


def lstm_unit(x_t, hidden_t_prev, cell_t_prev, forget_bias=0.0, param_attr=None, bias_attr=None, name=None):
    """fc([x, h_prev]) -> gates (i, f, o, g); c = f c_prev + i g, h = o tanh(c)  (lstm_unit_op.h)"""
    from .nn import fc
    D = T(hidden_t_prev).shape[-1]
    from ...tensor import concat
    g = fc(concat([x_t, hidden_t_prev], 1), 4 * D, param_attr=param_attr, bias_attr=bias_attr)
    return _lstm_unit_rec(g, cell_t_prev, D, forget_bias)


def _lstm_unit_run(g, cell_t_prev, D, forget_bias):
    i, f, o, gg = T(g).split(D, -1)
    c = torch.sigmoid(f + forget_bias) * T(cell_t_prev) + torch.sigmoid(i) * torch.tanh(gg)
    h = torch.sigmoid(o) * torch.tanh(c)
    return W(h), W(c)


_gru_unit_rec = static_op(_gru_unit_run, "gru_unit")
_lstm_unit_rec = static_op(_lstm_unit_run, "lstm_unit")


def lstm(input, init_h, init_c, max_len, hidden_size, num_layers, dropout_prob=0.0, is_bidirec=False,
         is_test=False, name=None, default_initializer=None, seed=-1):
    """multi-layer (bi)LSTM over time-major ``input`` [T, B, D] -> (out, last_h, last_c)"""
    x = T(input)
    net = _LSTM(x.shape[-1], hidden_size, num_layers, "bidirect" if is_bidirec else "forward", time_major=True,
                dropout=0.0 if is_test else dropout_prob)
    out, (h, c) = net(W(x), (init_h, init_c))
    return out, h, c


# ----------------------------------------------------------------------------- LoD beam search
def beam_search(pre_ids, pre_scores, ids, scores, beam_size, end_id, level=0, is_accumulated=True, name=None,
                return_parent_idx=False):
    """one beam-search step over LoD prefixes (beam_search_op.h): each source keeps the
    ``beam_size`` best (prefix, candidate) extensions; ended prefixes (pre_id == end_id) carry
    over alone. -> (selected_ids, selected_scores[, parent_idx]) with 2-level LoD
    [source -> prefixes, prefix -> selections]."""
    pi = T(pre_ids).reshape(-1).tolist()
    ps = T(pre_scores).reshape(-1).tolist()
    sc = T(scores)
    cand_ids = T(ids) if ids is not None else None
    lod = fcore.lod_of(pre_ids)
    src_off = lod[0] if lod else [0, len(pi)]
    if len(lod) > 1:
        # prefixes of source s are the rows of its level-1 range
        src_off = [lod[1][k] for k in lod[0]]
    K = sc.shape[-1]
    sel_ids, sel_sc, parents, per_prefix = [], [], [], [0] * len(pi)
    for s in range(len(src_off) - 1):
        cands = []
        for p in range(src_off[s], src_off[s + 1]):
            if pi[p] == end_id:
                cands.append((ps[p], p, end_id))
                continue
            for k in range(K):
                v = float(sc[p, k])
                tok = int(cand_ids[p, k]) if cand_ids is not None else k
                total = v if is_accumulated else ps[p] + float(torch.log(torch.tensor(v)))
                cands.append((total, p, tok))
        cands.sort(key=lambda c: (-c[0], c[1]))
        chosen = sorted(cands[:beam_size], key=lambda c: c[1])
        for v, p, tok in chosen:
            sel_ids.append(tok)
            sel_sc.append(v)
            parents.append(p)
            per_prefix[p] += 1
    n_src = [sum(1 for _ in range(src_off[s], src_off[s + 1])) for s in range(len(src_off) - 1)]
    l0 = fcore._offsets_from_lengths(n_src)
    l1 = fcore._offsets_from_lengths(per_prefix)
    oi = W(torch.tensor(sel_ids, dtype=torch.int64, device=dev())[:, None])
    os_ = W(torch.tensor(sel_sc, dtype=torch.float32, device=dev())[:, None])
    oi._lod = os_._lod = [l0, l1]
    if return_parent_idx:
        return oi, os_, W(torch.tensor(parents, dtype=torch.int64, device=dev()))
    return oi, os_


def beam_search_decode(ids, scores, beam_size, end_id, name=None):
    """back-trace the per-step selections (arrays of beam_search outputs) into full hypotheses:
    -> (sentence_ids, sentence_scores), LoD [source -> hypotheses, hypothesis -> tokens]"""
    steps = len(ids)
    # parent of selection j at step t = the prefix row (of step t-1) whose level-1 range holds j
    parents = []
    for t in range(steps):
        l1 = fcore.lod_of(ids[t])[1]
        par = []
        for p in range(len(l1) - 1):
            par += [p] * (l1[p + 1] - l1[p])
        parents.append(par)
    last = steps - 1
    l0 = fcore.lod_of(ids[0])[0]
    n_src = len(l0) - 1
    # hypotheses end at an end_id selection or at the last step
    hyps = [[] for _ in range(n_src)]
    for t in range(steps):
        idv = T(ids[t]).reshape(-1).tolist()
        scv = T(scores[t]).reshape(-1).tolist()
        lod_t = fcore.lod_of(ids[t])
        for j, tok in enumerate(idv):
            if tok == end_id or t == last:
                prev_ended = t > 0 and T(ids[t - 1]).reshape(-1).tolist()[parents[t][j]] == end_id
                if prev_ended:
                    continue
                seq, k = [], j
                for u in range(t, -1, -1):
                    seq.append(int(T(ids[u]).reshape(-1)[k]))
                    if u > 0:
                        k = parents[u][k]
                src = _source_of(lod_t, j)
                hyps[src].append((seq[::-1], scv[j]))
    flat_ids, flat_sc, n_h, lens = [], [], [], []
    for s in range(n_src):
        hs = sorted(hyps[s], key=lambda h: -h[1])[:beam_size]
        n_h.append(len(hs))
        for seq, v in hs:
            flat_ids += seq
            flat_sc += [v] * len(seq)
            lens.append(len(seq))
    oi = W(torch.tensor(flat_ids, dtype=torch.int64, device=dev())[:, None])
    os_ = W(torch.tensor(flat_sc, dtype=torch.float32, device=dev())[:, None])
    oi._lod = os_._lod = [fcore._offsets_from_lengths(n_h), fcore._offsets_from_lengths(lens)]
    return oi, os_


def _source_of(lod, j):
    l0, l1 = lod[0], lod[1]
    for s in range(len(l0) - 1):
        if l1[l0[s]] <= j < l1[l0[s + 1]]:
            return s
    return len(l0) - 2


_ = (Tensor, to_padded, from_padded)
