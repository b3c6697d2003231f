"""``fluid.layers`` losses (reference: python/paddle/fluid/layers/loss.py; op semantics from
paddle/fluid/operators/{cross_entropy,bpr_loss,center_loss,rank_loss,margin_rank_loss,
teacher_student_sigmoid_loss,sampled_softmax_with_cross_entropy...}_op.h). Per-sample losses
keep the reference's trailing unit dimension ([N, 1])."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as TF

from ...nn import functional as F
from ._common import T, W, dev, to_padded, register

__all__ = ["center_loss", "bpr_loss", "cross_entropy", "square_error_cost", "edit_distance", "warpctc", "nce",
           "hsigmoid", "sampled_softmax_with_cross_entropy", "softmax_with_cross_entropy", "rank_loss",
           "margin_rank_loss", "sigmoid_cross_entropy_with_logits", "teacher_student_sigmoid_loss", "huber_loss",
           "kldiv_loss", "npair_loss", "mse_loss"]

_BUILDERS = {"center_loss", "nce", "hsigmoid", "sampled_softmax_with_cross_entropy"}


def center_loss(input, label, num_classes, alpha, param_attr, update_center=True):
    """loss_i = ||x_i - c_{y_i}||^2 / 2; the centers move toward their samples by ``alpha`` times
    the mean difference (center_loss_op.h)"""
    from ._common import fparam as _create_parameter
    from ...nn import initializer as I
    x = T(input)
    centers = _create_parameter([num_classes, x.shape[1]], "float32", param_attr, default_initializer=I.Constant(0.0))
    y = T(label).reshape(-1).long()
    c = T(centers)
    diff = x - c[y]
    loss = 0.5 * (diff * diff).sum(1, keepdim=True)
    if update_center:
        with torch.no_grad():
            d = diff.detach()
            acc = torch.zeros_like(c).index_add_(0, y, d)
            cnt = torch.bincount(y, minlength=num_classes).to(c.dtype)[:, None]
            a = float(T(alpha).item()) if hasattr(alpha, "_t") else float(alpha)
            c.add_(a * acc / (1.0 + cnt))
    return W(loss)


def bpr_loss(input, label, name=None):
    """Bayesian personalised ranking: -mean_{j != y} log sigmoid(x_y - x_j), [N, 1]"""
    x = T(input)
    y = T(label).reshape(-1).long()
    pos = x.gather(1, y[:, None])
    lg = TF.logsigmoid(pos - x)
    mask = torch.ones_like(x).scatter_(1, y[:, None], 0.0)
    return W(-(lg * mask).sum(1, keepdim=True) / max(x.shape[1] - 1, 1))


def cross_entropy(input, label, soft_label=False, ignore_index=-100):
    """``input`` holds probabilities: hard labels -> -log p[label] (0 where label ==
    ignore_index), soft labels -> -sum(label * log p); shape [..., 1]"""
    p = T(input)
    if soft_label:
        return W(-(T(label) * torch.log(p)).sum(-1, keepdim=True))
    y = T(label).long()
    if y.dim() == p.dim():
        y = y.squeeze(-1)
    valid = y != ignore_index
    yy = torch.where(valid, y, torch.zeros_like(y))
    out = -torch.log(p.gather(-1, yy[..., None]))
    return W(out * valid[..., None].to(out.dtype))


def square_error_cost(input, label):
    d = T(input) - T(label)
    return W(d * d)


def _levenshtein(a, b):
    m, n = len(a), len(b)
    prev = list(range(n + 1))
    for i in range(1, m + 1):
        cur = [i] + [0] * n
        for j in range(1, n + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (a[i - 1] != b[j - 1]))
        prev = cur
    return prev[n]


def edit_distance(input, label, normalized=True, ignored_tokens=None, input_length=None, label_length=None):
    """(Levenshtein distance per sequence [N, 1] — divided by the label length when
    ``normalized`` — , number of sequences [1])"""
    x, xl, _ = to_padded(input, input_length)
    y, yl, _ = to_padded(label, label_length)
    x = x.reshape(x.shape[0], -1).tolist()
    y = y.reshape(y.shape[0], -1).tolist()
    ign = set(ignored_tokens or [])
    out = []
    for b in range(len(x)):
        a = [v for v in x[b][:int(xl[b])] if v not in ign]
        c = [v for v in y[b][:int(yl[b])] if v not in ign]
        d = float(_levenshtein(a, c))
        if normalized:
            d = d / max(len(c), 1)
        out.append([d])
    return W(torch.tensor(out, dtype=torch.float32, device=dev())), \
        W(torch.tensor([len(x)], dtype=torch.int64, device=dev()))


def warpctc(input, label, blank=0, norm_by_times=False, input_length=None, label_length=None):
    """CTC loss per sequence [N, 1] from unnormalised logits. Padded mode: ``input`` [T, N, C]
    with lengths; LoD mode: ``input`` [sum(T), C] and ``label`` [sum(L), 1] with LoD"""
    from .. import core as fcore
    if input_length is None:
        x, xl, _ = to_padded(input)
        x = x.transpose(0, 1)
        y, yl, _ = to_padded(label)
        y = y.reshape(y.shape[0], -1)
    else:
        x = T(input)
        xl = T(input_length).reshape(-1).long()
        y = T(label).reshape(T(label).shape[0], -1)
        yl = T(label_length).reshape(-1).long()
    lp = torch.log_softmax(x.float(), -1)
    loss = TF.ctc_loss(lp, y.long(), xl, yl, blank=blank, reduction="none", zero_infinity=False)
    if norm_by_times:
        loss = loss / xl.to(loss.dtype)
    _ = fcore
    return W(loss[:, None])


def nce(input, label, num_total_classes, sample_weight=None, param_attr=None, bias_attr=None, num_neg_samples=None,
        name=None, sampler="uniform", custom_dist=None, seed=0, is_sparse=False):
    from ...static import nn as SN
    return SN.nce(input, label, num_total_classes, sample_weight, param_attr, bias_attr, num_neg_samples, name,
                  sampler, custom_dist, seed, is_sparse)


def hsigmoid(input, label, num_classes, param_attr=None, bias_attr=None, name=None, path_table=None, path_code=None,
             is_custom=False, is_sparse=False):
    """hierarchical sigmoid over a complete binary tree (or a custom path table); creates the
    [num_classes - 1, D] weight and bias"""
    from ._common import fparam as _create_parameter
    d = T(input).shape[1]
    n = num_classes if is_custom else num_classes - 1
    w = _create_parameter([n, d], "float32", param_attr)
    b = None if bias_attr is False else _create_parameter([n, 1], "float32", bias_attr, is_bias=True)
    return F.hsigmoid_loss(input, label, num_classes, w, b, path_table, path_code, is_sparse)


def sampled_softmax_with_cross_entropy(logits, label, num_samples, num_true=1, remove_accidental_hits=True,
                                       use_customized_samples=False, customized_samples=None,
                                       customized_probabilities=None, seed=0):
    """softmax cross entropy over the true classes plus ``num_samples`` log-uniform negatives,
    logits corrected by -log Q (sample_logits_op.h); [N, 1]"""
    x = T(logits)
    N, K = x.shape
    y = T(label).reshape(N, -1).long()
    if use_customized_samples:
        samples = T(customized_samples).long()
        probs = T(customized_probabilities).to(x.dtype)
    else:
        g = np.random.RandomState(seed or None)
        # log-uniform (Zipf) sampler: P(k) = log((k + 2) / (k + 1)) / log(K + 1)
        u = g.uniform(size=num_samples)
        neg = np.clip(np.floor(np.exp(u * np.log(K + 1)) - 1).astype(np.int64), 0, K - 1)
        q = lambda k: np.log((k + 2.0) / (k + 1.0)) / np.log(K + 1.0)  # noqa: E731
        allc = np.concatenate([y.cpu().numpy(), np.broadcast_to(neg, (N, num_samples))], 1)
        samples = torch.from_numpy(allc).to(x.device)
        probs = torch.from_numpy(q(allc.astype(np.float64)) * num_samples).to(x.device, x.dtype)
    sl = x.gather(1, samples) - torch.log(probs)
    if remove_accidental_hits:
        hit = (samples[:, num_true:, None] == y[:, None, :]).any(-1)
        sl[:, num_true:] = sl[:, num_true:].masked_fill(hit, -1e20)
    lse = torch.logsumexp(sl, 1, keepdim=True)
    loss = -(sl[:, :num_true] - lse).sum(1, keepdim=True) / num_true
    return W(loss)


def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100, numeric_stable_mode=True,
                               return_softmax=False, axis=-1):
    return F.softmax_with_cross_entropy(logits, label, soft_label, ignore_index, numeric_stable_mode,
                                        return_softmax, axis)


def rank_loss(label, left, right, name=None):
    o = T(left) - T(right)
    return W(torch.log1p(torch.exp(o)) - T(label) * o)


def margin_rank_loss(label, left, right, margin=0.1, name=None):
    return W((-T(label) * (T(left) - T(right)) + margin).clamp_min(0))


def sigmoid_cross_entropy_with_logits(x, label, ignore_index=-100, name=None, normalize=False):
    t, y = T(x), T(label)
    loss = t.clamp_min(0) - t * y + torch.log1p(torch.exp(-t.abs()))
    valid = (y != ignore_index).to(loss.dtype)
    loss = loss * valid
    if normalize:
        loss = loss / valid.sum().clamp_min(1)
    return W(loss)


def teacher_student_sigmoid_loss(input, label, soft_max_up_bound=15.0, soft_max_lower_bound=-15.0):
    """label < -1: no teacher score, click 0; -1 <= label < 0: no teacher, click 1; 0 <= label
    < 1: teacher score z = label, click 0; label >= 1: z = label - 1, click 1
    (teacher_student_sigmoid_loss_op.h)"""
    x, y = T(input), T(label)
    base = x.clamp_min(0) + torch.log1p(torch.exp(-x.abs()))      # CE with target 0
    pos = base - x                                                 # CE with target 1
    out = torch.where(y < -1, base,
                      torch.where(y < 0, pos,
                                  torch.where(y < 1, base + base - x * y, pos + base - x * (y - 1))))
    return W(out)


def huber_loss(input, label, delta):
    r = T(label) - T(input)
    a = r.abs()
    return W(torch.where(a <= delta, 0.5 * r * r, delta * (a - 0.5 * delta)))


def kldiv_loss(x, target, reduction="mean", name=None):
    return F.kl_div(x, target, reduction)


def npair_loss(anchor, positive, labels, l2_reg=0.002):
    return F.npair_loss(anchor, positive, labels, l2_reg)


def mse_loss(input, label):
    d = T(input) - T(label)
    return W((d * d).mean())


register(globals(), __all__, skip=_BUILDERS)
