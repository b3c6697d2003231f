"""``fluid.layers.accuracy`` / ``auc`` (reference: python/paddle/fluid/layers/metric_op.py:33,131,
paddle/phi/kernels/cpu/auc_kernel.cc).

``auc`` keeps its statistics where the reference keeps them: in persistable int64 buffers created
with the layer (``batch_stat_pos / batch_stat_neg`` with the ``slide_steps`` ring and its step
counter, ``stat_pos / stat_neg`` for the global curve). In a static Program they are the Program's
persistable variables, updated in place by the two recorded ``auc`` ops at every run (two metrics in
one program, or two programs, never share state); in dygraph every call creates fresh buffers, as
the reference's ``create_global_variable`` does there."""
from __future__ import annotations

import torch

from ...framework import core as _core
from ...framework.dispatch import static_op
from ._common import T, W, dev

__all__ = ["accuracy", "auc"]


def accuracy(input, label, k=1, correct=None, total=None):
    """top-k accuracy [1] (fp32). In a static Program: the reference's two ops, top_k then
    accuracy on its indices (metric_op.py:33)"""
    from ...static.program import Variable, set_ref_op
    if _core._mode.static and isinstance(input, Variable):
        from ...tensor.search import topk
        vals, idx = topk(input, k)
        acc, c, t = _acc_rec(idx, label)
        set_ref_op(acc, "accuracy", {"Out": [vals], "Indices": [idx], "Label": [label]},
                   {"Accuracy": [acc], "Correct": [c], "Total": [t]}, {})
        return acc
    x = T(input)
    y = T(label).reshape(-1, 1).long()
    topk = torch.topk(x, k, -1).indices
    hit = (topk == y).any(-1)
    n_ok, n = int(hit.sum()), hit.numel()
    acc = W(torch.tensor([n_ok / max(n, 1)], dtype=torch.float32, device=dev()))
    if correct is not None:
        correct._t = torch.tensor([n_ok], dtype=torch.int32, device=dev())
    if total is not None:
        total._t = torch.tensor([n], dtype=torch.int32, device=dev())
    return acc


def _auc_area(pos, neg):
    """calcAuc: trapezoids over the thresholds from the highest bin down, / (P * N)"""
    tp = torch.flip(torch.cumsum(torch.flip(pos.double(), [0]), 0), [0])
    fp = torch.flip(torch.cumsum(torch.flip(neg.double(), [0]), 0), [0])
    tp_prev = torch.cat([tp[1:], tp.new_zeros(1)])
    fp_prev = torch.cat([fp[1:], fp.new_zeros(1)])
    area = ((fp - fp_prev).abs() * (tp + tp_prev) / 2).sum()
    P, N = tp[0], fp[0]
    return torch.where((P > 0) & (N > 0), area / (P * N).clamp_min(1), area).reshape(1)


def auc_op(predict, label, stat_pos, stat_neg, num_thresholds=2 ** 12 - 1, slide_steps=1, curve="ROC"):
    """the reference ``auc`` op: bins the positive-class probability (the last column) into
    ``num_thresholds + 1`` buckets, accumulates positives / negatives into the int64 stat buffers
    IN PLACE (``slide_steps`` > 0: a ring of per-step buckets plus their running sum, the step
    index in the last element) and returns the AUC of the accumulated counts (float64 [1]);
    ``curve`` is accepted and, as in auc_kernel.cc, the area is the ROC one"""
    p = T(predict)
    p = p.reshape(p.shape[0], -1)[:, -1]
    if bool(((p < 0) | (p > 1)).any()):
        raise ValueError("auc: the predict data must be in [0, 1]")
    y = T(label).reshape(-1)
    nb = num_thresholds + 1
    bins = (p.double() * num_thresholds).long().clamp(0, num_thresholds)
    cpos = torch.bincount(bins[y > 0], minlength=nb)
    cneg = torch.bincount(bins[y == 0], minlength=nb)
    sp, sn = T(stat_pos).reshape(-1), T(stat_neg).reshape(-1)
    with torch.no_grad():
        if slide_steps == 0:
            sp[:nb] += cpos.to(sp.device)
            sn[:nb] += cneg.to(sn.device)
            off = 0
        else:
            cur = int(sp[(slide_steps + 1) * nb]) % slide_steps
            c0, s0 = cur * nb, slide_steps * nb
            sp[s0:s0 + nb] -= sp[c0:c0 + nb]
            sn[s0:s0 + nb] -= sn[c0:c0 + nb]
            sp[c0:c0 + nb] = cpos.to(sp.device)
            sn[c0:c0 + nb] = cneg.to(sn.device)
            sp[s0:s0 + nb] += sp[c0:c0 + nb]
            sn[s0:s0 + nb] += sn[c0:c0 + nb]
            off = s0
        a = _auc_area(sp[off:off + nb], sn[off:off + nb])
        if slide_steps:
            sp[(slide_steps + 1) * nb] += 1
            sn[(slide_steps + 1) * nb] += 1
    return W(a.to(dev()))


_auc_rec = static_op(auc_op, "auc")


def _acc_run(indices, label):
    from ...static.ref_ops import accuracy_op
    return accuracy_op(indices, label)


_acc_rec = static_op(_acc_run, "accuracy")
_auc_counter = [0]


def _stat_buffer(shape, tag):
    t = W(torch.zeros(shape, dtype=torch.int64, device=dev()))
    t.persistable = True
    _auc_counter[0] += 1
    t.name = f"_generated_var_auc_{tag}_{_auc_counter[0]}"
    return t


def auc(input, label, curve="ROC", num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1):
    """(global AUC, batch AUC over the last ``slide_steps`` steps, [batch_stat_pos, batch_stat_neg,
    stat_pos, stat_neg]) — metric_op.py:131"""
    nb = num_thresholds + 1
    batch_pos = _stat_buffer([(1 + slide_steps) * nb + 1], "batch_stat_pos")
    batch_neg = _stat_buffer([(1 + slide_steps) * nb + 1], "batch_stat_neg")
    stat_pos = _stat_buffer([1, nb], "stat_pos")
    stat_neg = _stat_buffer([1, nb], "stat_neg")
    from ...static.program import set_ref_op
    outs = []
    for sp, sn, ss in ((batch_pos, batch_neg, slide_steps), (stat_pos, stat_neg, 0)):
        a = _auc_rec(input, label, sp, sn, num_thresholds=num_thresholds, slide_steps=ss, curve=curve)
        set_ref_op(a, "auc", {"Predict": [input], "Label": [label], "StatPos": [sp], "StatNeg": [sn]},
                   {"AUC": [a], "StatPosOut": [sp], "StatNegOut": [sn]},
                   {"curve": curve, "num_thresholds": int(num_thresholds), "slide_steps": int(ss)})
        outs.append(a)
    batch_auc, global_auc = outs
    return global_auc, batch_auc, [batch_pos, batch_neg, stat_pos, stat_neg]
