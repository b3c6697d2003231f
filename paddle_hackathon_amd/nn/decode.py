"""Decoding utilities (reference: python/paddle/fluid/layers/rnn.py: BeamSearchDecoder, dynamic_decode)."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap

__all__ = ["BeamSearchDecoder", "dynamic_decode", "Decoder"]


class Decoder:
    def initialize(self, inits):
        raise NotImplementedError

    def step(self, time, inputs, states, **kwargs):
        raise NotImplementedError

    def finalize(self, outputs, final_states, sequence_lengths):
        return outputs, final_states

    @property
    def tracks_own_finished(self):
        return False


def _map(fn, s):
    if isinstance(s, (list, tuple)):
        return type(s)(_map(fn, x) for x in s)
    if isinstance(s, Tensor):
        return _wrap(fn(s._t))
    return s


class BeamSearchDecoder(Decoder):
    """Beam search over a cell whose output is projected to vocab logits by ``output_fn``."""

    def __init__(self, cell, start_token, end_token, beam_size, embedding_fn=None, output_fn=None):
        self.cell, self.start_token, self.end_token = cell, start_token, end_token
        self.beam_size, self.embedding_fn, self.output_fn = beam_size, embedding_fn, output_fn

    @staticmethod
    def tile_beam_merge_with_batch(x, beam_size):
        t = x._t
        t = t.unsqueeze(1).expand(t.shape[0], beam_size, *t.shape[1:])
        return _wrap(t.reshape(-1, *t.shape[2:]))

    def _merge(self, t):
        return t.reshape(-1, *t.shape[2:])

    def _split(self, t):
        return t.reshape(-1, self.beam_size, *t.shape[1:])

    def initialize(self, initial_cell_states):
        def first(s):
            while isinstance(s, (list, tuple)):
                s = s[0]
            return s
        b = first(initial_cell_states)._t.shape[0]
        dev = first(initial_cell_states)._t.device
        self.batch_size = b
        states = _map(lambda t: t.unsqueeze(1).expand(b, self.beam_size, *t.shape[1:]).reshape(b * self.beam_size, *t.shape[1:]).contiguous(),
                      initial_cell_states)
        log_probs = torch.full((b, self.beam_size), float("-inf"), device=dev)
        log_probs[:, 0] = 0.0
        finished = torch.zeros(b, self.beam_size, dtype=torch.bool, device=dev)
        lengths = torch.zeros(b, self.beam_size, dtype=torch.int64, device=dev)
        ids = torch.full((b * self.beam_size,), self.start_token, dtype=torch.int64, device=dev)
        inputs = self.embedding_fn(_wrap(ids)) if self.embedding_fn else _wrap(ids)
        return inputs, (states, log_probs, finished, lengths), finished

    def step(self, time, inputs, states, **kwargs):
        cell_states, log_probs, finished, lengths = states
        out, new_cell = self.cell(inputs, cell_states, **kwargs)
        logits = self.output_fn(out) if self.output_fn else out
        lp = torch.log_softmax(logits._t.float(), -1)
        V = lp.shape[-1]
        lp = lp.reshape(self.batch_size, self.beam_size, V)
        # finished beams only extend with end_token at zero cost
        fin_mask = torch.full((V,), float("-inf"), device=lp.device)
        fin_mask[self.end_token] = 0.0
        lp = torch.where(finished.unsqueeze(-1), fin_mask.expand_as(lp), lp)
        scores = (log_probs.unsqueeze(-1) + lp).reshape(self.batch_size, -1)
        top, idx = torch.topk(scores, self.beam_size, -1)
        beam_idx = idx // V
        token = idx % V
        gather = (beam_idx + torch.arange(self.batch_size, device=lp.device).unsqueeze(1) * self.beam_size).reshape(-1)
        new_cell = _map(lambda t: t[gather], new_cell)
        prev_fin = torch.gather(finished, 1, beam_idx)
        new_fin = prev_fin | (token == self.end_token)
        new_len = torch.gather(lengths, 1, beam_idx) + (~prev_fin).long()
        ids = token.reshape(-1)
        nxt = self.embedding_fn(_wrap(ids)) if self.embedding_fn else _wrap(ids)
        outputs = (_wrap(top), _wrap(token), _wrap(beam_idx))
        return outputs, (new_cell, top, new_fin, new_len), nxt, new_fin

    def finalize(self, outputs, final_states, sequence_lengths):
        scores, tokens, parents = outputs
        T = tokens.shape[0]
        ids = tokens.clone()
        par = parents[T - 1]
        for t in range(T - 2, -1, -1):
            ids[t] = torch.gather(tokens[t], 1, par)
            par = torch.gather(parents[t], 1, par)
        ids[T - 1] = tokens[T - 1]
        return _wrap(ids), final_states


def dynamic_decode(decoder, inits=None, max_step_num=None, output_time_major=False, impute_finished=False,
                   is_test=False, return_length=False, **kwargs):
    inputs, states, finished = decoder.initialize(inits)
    outs = []
    step = 0
    while True:
        o, states, inputs, finished = decoder.step(step, inputs, states, **kwargs)
        outs.append(tuple(x._t for x in o) if isinstance(o, tuple) else o._t)
        step += 1
        if bool(finished.all()) or (max_step_num is not None and step > max_step_num):
            break
    if isinstance(outs[0], tuple):
        stacked = tuple(torch.stack([o[i] for o in outs], 0) for i in range(len(outs[0])))
    else:
        stacked = torch.stack(outs, 0)
    lengths = states[3] if isinstance(states, tuple) and len(states) == 4 else None
    final, fstates = decoder.finalize(stacked, states, lengths)
    ft = final._t
    if not output_time_major:
        ft = ft.transpose(0, 1)
    res = (_wrap(ft), fstates)
    if return_length:
        res = res + (_wrap(lengths) if lengths is not None else None,)
    return res
