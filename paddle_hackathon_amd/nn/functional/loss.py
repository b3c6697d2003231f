"""Losses (reference: python/paddle/nn/functional/loss.py,
phi/kernels/gpu/cross_entropy_kernel.cu). Hard-label softmax cross-entropy on
HIP tensors runs the fused one-pass gfx950 kernel (ops.softmax_cross_entropy)."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops
from ... import ops as _ops

_w = _wrap


def _up(t):
    """Compute losses in fp32 for half inputs, at input precision otherwise (fp64 stays fp64)."""
    return t.float() if t.dtype in (torch.float16, torch.bfloat16) else t


__all__ = ["binary_cross_entropy", "binary_cross_entropy_with_logits", "cross_entropy", "softmax_with_cross_entropy",
           "ctc_loss", "dice_loss", "hinge_embedding_loss", "hsigmoid_loss", "kl_div", "l1_loss", "log_loss",
           "margin_ranking_loss", "mse_loss", "nll_loss", "npair_loss", "sigmoid_focal_loss", "smooth_l1_loss",
           "square_error_cost", "cosine_embedding_loss", "margin_cross_entropy", "multi_label_soft_margin_loss",
           "soft_margin_loss", "triplet_margin_loss", "triplet_margin_with_distance_loss", "poisson_nll_loss",
           "gaussian_nll_loss", "multi_margin_loss", "identity_loss"]


def _t(x):
    return None if x is None else (x._t if isinstance(x, Tensor) else x)


def _reduce(loss, reduction):
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss


def cross_entropy(input, label, weight=None, ignore_index=-100, reduction="mean", soft_label=False, axis=-1,
                  use_softmax=True, name=None, label_smoothing=0.0):
    x = input._t
    lab = label._t
    axis = axis % x.dim()
    if soft_label:
        logp = TF.log_softmax(_up(x), axis) if use_softmax else torch.log(_up(x))
        lf = lab.to(logp.dtype)
        loss = -(lf * logp).sum(axis, keepdim=True)
        if weight is not None:
            # reference (test_cross_entropy_loss.py cross_entropy_soft): each sample's loss is
            # scaled by dot(weight, its soft label) and 'mean' divides by the sum of those weights
            shape = [1] * x.dim()
            shape[axis] = -1
            cw = (lf * _t(weight).to(logp.dtype).reshape(shape)).sum(axis, keepdim=True)
            loss = loss * cw
            if reduction == "mean":
                return _w(loss.sum() / cw.sum())
        return _w(_reduce(loss, reduction))
    if lab.dim() == x.dim():
        lab = lab.squeeze(axis)
    lab = lab.long()
    if axis != x.dim() - 1:
        x = x.movedim(axis, -1)
    if use_softmax and weight is None and label_smoothing == 0.0:
        loss = _ops.softmax_cross_entropy(x, lab, ignore_index)
        if reduction == "mean":
            valid = (lab != ignore_index).sum().clamp_min(1)
            return _w(loss.sum() / valid)
        if reduction == "sum":
            return _w(loss.sum())
        return _w(loss.unsqueeze(-1) if axis == input._t.dim() - 1 else loss)
    logp = TF.log_softmax(_up(x), -1) if use_softmax else torch.log(_up(x))
    C = logp.shape[-1]
    flat = logp.reshape(-1, C)
    lf = lab.reshape(-1)
    w = _t(weight)
    loss = TF.nll_loss(flat, lf, weight=None if w is None else w.to(flat.dtype), ignore_index=ignore_index,
                       reduction="none")
    if label_smoothing:
        smooth = -flat.mean(-1)
        loss = (1 - label_smoothing) * loss + label_smoothing * smooth
    if reduction == "mean":
        if w is not None:
            valid = lf != ignore_index
            den = w.to(flat.dtype)[lf.clamp_min(0)] * valid
            return _w(loss.sum() / den.sum())
        valid = (lf != ignore_index).sum().clamp_min(1)
        return _w(loss.sum() / valid)
    if reduction == "sum":
        return _w(loss.sum())
    return _w(loss.reshape(lab.shape).unsqueeze(-1))


def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100, numeric_stable_mode=True,
                               return_softmax=False, axis=-1):
    x = logits._t
    axis = axis % x.dim()
    if soft_label:
        logp = TF.log_softmax(_up(x), axis)
        loss = -(label._t.to(logp.dtype) * logp).sum(axis, keepdim=True)
    else:
        lab = label._t
        if lab.dim() == x.dim():
            lab = lab.squeeze(axis)
        xm = x.movedim(axis, -1) if axis != x.dim() - 1 else x
        loss = _ops.softmax_cross_entropy(xm, lab.long(), ignore_index).unsqueeze(-1)
        if axis != x.dim() - 1:
            loss = loss.movedim(-1, axis)
    loss = loss.to(x.dtype) if x.dtype == torch.float64 else loss
    if return_softmax:
        return _w(loss), _w(torch.softmax(x, axis))
    return _w(loss)


def binary_cross_entropy(input, label, weight=None, reduction="mean", name=None):
    return _w(TF.binary_cross_entropy(input._t, label._t, weight=_t(weight), reduction=reduction))


def binary_cross_entropy_with_logits(logit, label, weight=None, reduction="mean", pos_weight=None, name=None):
    return _w(TF.binary_cross_entropy_with_logits(logit._t, label._t, weight=_t(weight), reduction=reduction,
                                                  pos_weight=_t(pos_weight)))


def ctc_loss(log_probs, labels, input_lengths, label_lengths, blank=0, reduction="mean", norm_by_times=False):
    lp = TF.log_softmax(log_probs._t.float(), -1)
    loss = TF.ctc_loss(lp, labels._t, input_lengths._t, label_lengths._t, blank, reduction="none", zero_infinity=True)
    if reduction == "mean":
        return _w((loss / label_lengths._t.clamp_min(1).float()).mean())
    return _w(_reduce(loss, reduction))


def dice_loss(input, label, epsilon=0.00001, name=None):
    x = input._t
    lab = TF.one_hot(label._t.squeeze(-1).long(), x.shape[-1]).to(x.dtype)
    dims = tuple(range(1, x.dim()))
    inter = (x * lab).sum(dims)
    union = x.sum(dims) + lab.sum(dims)
    return _w((1 - (2 * inter) / (union + epsilon)).mean())


def hinge_embedding_loss(input, label, margin=1.0, reduction="mean", name=None):
    return _w(TF.hinge_embedding_loss(input._t, label._t, margin, reduction=reduction))


def hsigmoid_loss(input, label, num_classes, weight, bias=None, path_table=None, path_code=None, is_sparse=False, name=None):
    # default complete binary tree coding (reference: phi/kernels/funcs/matrix_bit_code.h)
    x = input._t
    lab = label._t.reshape(-1).long()
    w = weight._t
    code_len = int(num_classes - 1).bit_length()
    losses = []
    c = lab + num_classes
    out = torch.zeros(x.shape[0], device=x.device, dtype=torch.float32)
    for j in range(code_len):
        idx = (c >> (j + 1)) - 1
        bit = ((c >> j) & 1).float()
        valid = (c >> (j + 1)) > 0
        idx_c = idx.clamp_min(0)
        pre = (x.float() * w[idx_c].float()).sum(-1)
        if bias is not None:
            pre = pre + bias._t.reshape(-1)[idx_c].float()
        l = TF.binary_cross_entropy_with_logits(pre, bit, reduction="none")
        out = out + torch.where(valid, l, torch.zeros_like(l))
    return _w(out.unsqueeze(-1))


def kl_div(input, label, reduction="mean", name=None):
    x, y = input._t, label._t
    loss = y * (torch.log(y.clamp_min(1e-38)) - x)
    loss = torch.where(y > 0, loss, torch.zeros_like(loss))
    if reduction == "batchmean":
        return _w(loss.sum() / x.shape[0])
    return _w(_reduce(loss, reduction))


def l1_loss(input, label, reduction="mean", name=None):
    return _w(TF.l1_loss(input._t, label._t, reduction=reduction))


def log_loss(input, label, epsilon=0.0001, name=None):
    x, y = input._t, label._t
    return _w(-y * torch.log(x + epsilon) - (1 - y) * torch.log(1 - x + epsilon))


def margin_ranking_loss(input, other, label, margin=0.0, reduction="mean", name=None):
    return _w(TF.margin_ranking_loss(input._t, other._t, label._t, margin, reduction=reduction))


def mse_loss(input, label, reduction="mean", name=None):
    return _w(TF.mse_loss(input._t, label._t, reduction=reduction))


def square_error_cost(input, label):
    return _w((input._t - label._t) ** 2)


def nll_loss(input, label, weight=None, ignore_index=-100, reduction="mean", name=None):
    x = input._t
    lab = label._t.long()
    if x.dim() > 2:
        x = x.movedim(1, -1).reshape(-1, x.shape[1])
        lab = lab.reshape(-1)
        out = TF.nll_loss(x, lab, _t(weight), ignore_index=ignore_index, reduction=reduction)
        if reduction == "none":
            out = out.reshape(label._t.shape)
        return _w(out)
    return _w(TF.nll_loss(x, lab, _t(weight), ignore_index=ignore_index, reduction=reduction))


def npair_loss(anchor, positive, labels, l2_reg=0.002):
    a, p, lab = anchor._t, positive._t, labels._t.reshape(-1, 1).float()
    reg = l2_reg * ((a ** 2).sum(1).mean() + (p ** 2).sum(1).mean()) * 0.25
    same = (lab == lab.t()).float()
    same = same / same.sum(1, keepdim=True)
    logits = a @ p.t()
    ce = (-same * TF.log_softmax(logits, 1)).sum(1).mean()
    return _w(ce + reg)


def sigmoid_focal_loss(logit, label, normalizer=None, alpha=0.25, gamma=2.0, reduction="sum", name=None):
    x, y = logit._t, label._t
    p = torch.sigmoid(x)
    ce = TF.binary_cross_entropy_with_logits(x, y, reduction="none")
    p_t = p * y + (1 - p) * (1 - y)
    loss = ce * ((1 - p_t) ** gamma)
    if alpha >= 0:
        loss = (alpha * y + (1 - alpha) * (1 - y)) * loss
    if normalizer is not None:
        loss = loss / normalizer._t
    return _w(_reduce(loss, reduction))


def smooth_l1_loss(input, label, reduction="mean", delta=1.0, name=None):
    return _w(TF.huber_loss(input._t, label._t, reduction=reduction, delta=delta))


def cosine_embedding_loss(input1, input2, label, margin=0, reduction="mean", name=None):
    return _w(TF.cosine_embedding_loss(input1._t, input2._t, label._t, margin, reduction=reduction))


class _ReplicatedSum(torch.autograd.Function):
    """all-reduce SUM whose backward is the identity: every rank goes on with the same replicated
    value and backpropagates it, so each rank's local partial receives the gradient once (the
    model-parallel reduce rule; torch's autograd all_reduce would sum the replicas' gradients)"""

    @staticmethod
    def forward(ctx, x, pg):
        import torch.distributed as tdist
        y = x.clone()
        tdist.all_reduce(y, op=tdist.ReduceOp.SUM, group=pg)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


def margin_cross_entropy(logits, label, margin1=1.0, margin2=0.5, margin3=0.0, scale=64.0, group=None,
                         return_softmax=False, reduction="mean"):
    """ArcFace-style margin softmax cross-entropy (reference nn/functional/loss.py
    margin_cross_entropy + the margin_cross_entropy kernel). Class-parallel like the reference:
    with a distributed job (``group`` None = the default group, or a Group; ``group=False`` forces
    the single-rank form) every rank holds its shard of the class dimension, labels are global
    class ids, and the softmax normaliser is reduced over the group (max, then sum of exp) —
    the returned softmax is this rank's shard of the global one."""
    import torch.distributed as tdist
    x = _up(logits._t)
    lab = label._t.reshape(-1).long()
    pg, nranks = None, 1
    if group is not False and tdist.is_available() and tdist.is_initialized():
        pg = getattr(group, "process_group", None) if group is not None else None
        nranks = tdist.get_world_size(pg) if (group is None or pg is not None) else 1
    C = x.shape[-1]
    start = 0
    if nranks > 1:
        counts = [torch.zeros(1, dtype=torch.int64, device=x.device) for _ in range(nranks)]
        tdist.all_gather(counts, torch.tensor([C], dtype=torch.int64, device=x.device), group=pg)
        me = tdist.get_rank(pg)
        start = int(sum(int(c.item()) for c in counts[:me]))
    local = lab - start
    own = (local >= 0) & (local < C)
    theta = torch.acos(x.clamp(-1 + 1e-7, 1 - 1e-7))
    tgt = torch.cos(margin1 * theta + margin2) - margin3
    oh = TF.one_hot(local.clamp(0, C - 1), C).bool() & own[:, None]
    adj = torch.where(oh, tgt, x) * scale
    if nranks == 1:
        loss = TF.cross_entropy(adj, lab, reduction="none").unsqueeze(-1)
        sm = torch.softmax(adj, -1) if return_softmax else None
    else:
        m = adj.detach().max(-1, keepdim=True).values
        tdist.all_reduce(m, op=tdist.ReduceOp.MAX, group=pg)
        e = torch.exp(adj - m)
        ssum = _ReplicatedSum.apply(e.sum(-1, keepdim=True), pg)
        t = _ReplicatedSum.apply((adj - m).masked_fill(~oh, 0.0).sum(-1, keepdim=True), pg)
        loss = torch.log(ssum) - t
        sm = e / ssum if return_softmax else None
    loss = _reduce(loss, reduction) if reduction else loss
    if return_softmax:
        return _w(loss), _w(sm)
    return _w(loss)


def multi_label_soft_margin_loss(input, label, weight=None, reduction="mean", name=None):
    return _w(TF.multilabel_soft_margin_loss(input._t, label._t, weight=_t(weight), reduction=reduction))


def soft_margin_loss(input, label, reduction="mean", name=None):
    return _w(TF.soft_margin_loss(input._t, label._t.to(input._t.dtype), reduction=reduction))


def triplet_margin_loss(input, positive, negative, margin=1.0, p=2, epsilon=1e-6, swap=False, reduction="mean", name=None):
    return _w(TF.triplet_margin_loss(input._t, positive._t, negative._t, margin, p, epsilon, swap, reduction=reduction))


def triplet_margin_with_distance_loss(input, positive, negative, distance_function=None, margin=1.0, swap=False,
                                      reduction="mean", name=None):
    df = None
    if distance_function is not None:
        def df(a, b):
            return _t(distance_function(_w(a), _w(b)))
    return _w(TF.triplet_margin_with_distance_loss(input._t, positive._t, negative._t, distance_function=df,
                                                   margin=margin, swap=swap, reduction=reduction))


def poisson_nll_loss(input, label, log_input=True, full=False, epsilon=1e-8, reduction="mean", name=None):
    return _w(TF.poisson_nll_loss(input._t, label._t, log_input, full, eps=epsilon, reduction=reduction))


def gaussian_nll_loss(input, label, variance, full=False, epsilon=1e-6, reduction="mean", name=None):
    return _w(TF.gaussian_nll_loss(input._t, label._t, variance._t, full, epsilon, reduction))


def multi_margin_loss(input, label, p=1, margin=1.0, weight=None, reduction="mean", name=None):
    return _w(TF.multi_margin_loss(input._t, label._t, p, margin, _t(weight), reduction=reduction))


def identity_loss(x, reduction="none"):
    if reduction in (0, "sum"):
        return _w(x._t.sum())
    if reduction in (1, "mean"):
        return _w(x._t.mean())
    return x


register_ops(globals(), __all__)
