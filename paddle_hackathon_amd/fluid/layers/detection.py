"""``fluid.layers`` detection ops (reference: python/paddle/fluid/layers/detection.py; kernels
paddle/fluid/operators/detection/*_op.{h,cc}). Box ops run on device tensors; the matching,
sampling and NMS stages are per-image host loops, as in the reference's CPU kernels (their
outputs have data-dependent sizes)."""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as TF

from ...vision import ops as V
from ...static import nn as SN
from ._common import T, W, dev, register
from .. import core as fcore

__all__ = ["prior_box", "density_prior_box", "multi_box_head", "bipartite_match", "target_assign",
           "detection_output", "ssd_loss", "rpn_target_assign", "retinanet_target_assign", "sigmoid_focal_loss",
           "anchor_generator", "roi_perspective_transform", "generate_proposal_labels", "generate_proposals",
           "generate_mask_labels", "iou_similarity", "box_coder", "polygon_box_transform", "yolov3_loss", "yolo_box",
           "box_clip", "multiclass_nms", "locality_aware_nms", "matrix_nms", "retinanet_detection_output",
           "distribute_fpn_proposals", "box_decoder_and_assign", "collect_fpn_proposals"]


def _iou(a, b, normalized=True):
    off = 0.0 if normalized else 1.0
    aw = (a[:, 2] - a[:, 0] + off).clamp_min(0)
    ah = (a[:, 3] - a[:, 1] + off).clamp_min(0)
    bw = (b[:, 2] - b[:, 0] + off).clamp_min(0)
    bh = (b[:, 3] - b[:, 1] + off).clamp_min(0)
    x1 = torch.maximum(a[:, None, 0], b[None, :, 0])
    y1 = torch.maximum(a[:, None, 1], b[None, :, 1])
    x2 = torch.minimum(a[:, None, 2], b[None, :, 2])
    y2 = torch.minimum(a[:, None, 3], b[None, :, 3])
    inter = (x2 - x1 + off).clamp_min(0) * (y2 - y1 + off).clamp_min(0)
    union = aw[:, None] * ah[:, None] + bw[None] * bh[None] - inter
    return torch.where(union > 0, inter / union, torch.zeros_like(inter))


def _offsets(x, n_rows=None):
    lod = fcore.lod_of(x)
    if lod:
        return lod[-1]
    return [0, n_rows if n_rows is not None else T(x).shape[0]]


def _lod_out(t, lens):
    o = W(t)
    o._lod = [fcore._offsets_from_lengths(lens)]
    return o


# ----------------------------------------------------------------------------- priors / anchors
def prior_box(input, image, min_sizes, max_sizes=None, aspect_ratios=[1.0], variance=[0.1, 0.1, 0.2, 0.2],
              flip=False, clip=False, steps=[0.0, 0.0], offset=0.5, name=None, min_max_aspect_ratios_order=False):
    return V.prior_box(input, image, min_sizes, max_sizes, aspect_ratios, variance, flip, clip, steps, offset,
                       min_max_aspect_ratios_order)


def density_prior_box(input=None, image=None, densities=None, fixed_sizes=None, fixed_ratios=None,
                      variance=[0.1, 0.1, 0.2, 0.2], clip=False, steps=[0.0, 0.0], offset=0.5, flatten_to_2d=False,
                      name=None):
    H, Wd = T(input).shape[2:]
    IH, IW = T(image).shape[2:]
    sw = steps[0] or IW / Wd
    sh = steps[1] or IH / H
    step_avg = int((sw + sh) * 0.5)
    boxes = []
    for h in range(H):
        for w in range(Wd):
            cx, cy = (w + offset) * sw, (h + offset) * sh
            for size, dens in zip(fixed_sizes, densities):
                shift = step_avg // dens
                for r in fixed_ratios:
                    bw, bh = size * math.sqrt(r), size / math.sqrt(r)
                    dcx = cx - step_avg / 2.0 + shift / 2.0
                    dcy = cy - step_avg / 2.0 + shift / 2.0
                    for di in range(dens):
                        for dj in range(dens):
                            x, y = dcx + dj * shift, dcy + di * shift
                            boxes.append([max((x - bw / 2) / IW, 0.0), max((y - bh / 2) / IH, 0.0),
                                          min((x + bw / 2) / IW, 1.0), min((y + bh / 2) / IH, 1.0)])
    b = torch.tensor(boxes, dtype=torch.float32, device=dev()).reshape(H, Wd, -1, 4)
    if clip:
        b = b.clamp(0, 1)
    v = torch.tensor(variance, dtype=torch.float32, device=b.device).expand_as(b).contiguous()
    if flatten_to_2d:
        return W(b.reshape(-1, 4)), W(v.reshape(-1, 4))
    return W(b), W(v)


def anchor_generator(input, anchor_sizes=None, aspect_ratios=None, variance=[0.1, 0.1, 0.2, 0.2], stride=None,
                     offset=0.5, name=None):
    """-> (anchors [H, W, A, 4], variances [H, W, A, 4]); A = len(ratios) * len(sizes), ratios
    outer (anchor_generator_op.h)"""
    H, Wd = T(input).shape[2:]
    sizes = anchor_sizes if isinstance(anchor_sizes, (list, tuple)) else [anchor_sizes]
    ratios = aspect_ratios if isinstance(aspect_ratios, (list, tuple)) else [aspect_ratios]
    sw, sh = float(stride[0]), float(stride[1])
    base = []
    for ar in ratios:
        for s in sizes:
            area_ratio = (sw * sh) / ar
            bw = round(math.sqrt(area_ratio))
            bh = round(bw * ar)
            base.append((s / sw * bw, s / sh * bh))
    xs = torch.arange(Wd, dtype=torch.float32) * sw + offset * (sw - 1)
    ys = torch.arange(H, dtype=torch.float32) * sh + offset * (sh - 1)
    cy, cx = torch.meshgrid(ys, xs, indexing="ij")
    wh = torch.tensor(base, dtype=torch.float32)
    a = torch.stack([cx[..., None] - 0.5 * (wh[:, 0] - 1), cy[..., None] - 0.5 * (wh[:, 1] - 1),
                     cx[..., None] + 0.5 * (wh[:, 0] - 1), cy[..., None] + 0.5 * (wh[:, 1] - 1)], -1).to(dev())
    v = torch.tensor(variance, dtype=torch.float32, device=a.device).expand_as(a).contiguous()
    return W(a), W(v)


def multi_box_head(inputs, image, base_size, num_classes, aspect_ratios, min_ratio=None, max_ratio=None,
                   min_sizes=None, max_sizes=None, steps=None, step_w=None, step_h=None, offset=0.5,
                   variance=[0.1, 0.1, 0.2, 0.2], flip=True, clip=False, kernel_size=1, pad=0, stride=1, name=None,
                   min_max_aspect_ratios_order=False):
    return SN.multi_box_head(inputs, image, base_size, num_classes, aspect_ratios, min_ratio, max_ratio, min_sizes,
                             max_sizes, steps, step_w, step_h, offset, variance, flip, clip, kernel_size, pad, stride,
                             name, min_max_aspect_ratios_order)


# ----------------------------------------------------------------------------- matching
def iou_similarity(x, y, box_normalized=True, name=None):
    out = _iou(T(x).float(), T(y).float(), box_normalized)
    return W(out, x)


def _bipartite(d, match_type, thr):
    K, M = d.shape
    idx = np.full(M, -1, dtype=np.int64)
    dist = np.zeros(M, dtype=np.float32)
    dd = d.copy()
    row_used = np.zeros(K, bool)
    for _ in range(min(K, M)):
        flat = np.where(row_used[:, None] | (idx[None, :] >= 0), -1.0, dd)
        k = int(np.argmax(flat))
        r, c = divmod(k, M)
        if flat[r, c] <= 0:     # only positive similarities match (bipartite_match_op.cc)
            break
        idx[c], dist[c], row_used[r] = r, d[r, c], True
    if match_type == "per_prediction":
        t = 0.5 if thr is None else thr
        for c in range(M):
            if idx[c] < 0 and K:
                r = int(np.argmax(d[:, c]))
                if d[r, c] >= t:
                    idx[c], dist[c] = r, d[r, c]
    return idx, dist


def bipartite_match(dist_matrix, match_type=None, dist_threshold=None, name=None):
    """greedy bipartite matching of ground-truth rows to prior columns per image (rows split by
    the LoD); -> (match_indices [N, M] int32, -1 unmatched; match_distance [N, M])"""
    d = T(dist_matrix).float().cpu().numpy()
    off = _offsets(dist_matrix, d.shape[0])
    idxs, dists = [], []
    for a, b in zip(off[:-1], off[1:]):
        i, s = _bipartite(d[a:b], match_type, dist_threshold)
        idxs.append(i)
        dists.append(s)
    return W(torch.from_numpy(np.stack(idxs).astype(np.int32)).to(dev())), \
        W(torch.from_numpy(np.stack(dists)).to(dev()))


def target_assign(input, matched_indices, negative_indices=None, mismatch_value=None, name=None):
    """out[i, j] = input[lod[i] + match[i, j], j] (or mismatch_value); weight 1 where matched
    or listed as negative (target_assign_op.h)"""
    x = T(input)
    m = T(matched_indices).long()
    off = _offsets(input, x.shape[0])
    N, P = m.shape
    K = x.shape[-1]
    mv = 0.0 if mismatch_value is None else float(mismatch_value)
    out = torch.full((N, P, K), mv, dtype=x.dtype, device=x.device)
    wt = torch.zeros((N, P, 1), dtype=torch.float32, device=x.device)
    for i in range(N):
        sel = m[i] >= 0
        cols = torch.nonzero(sel).reshape(-1)
        if cols.numel():
            rows = off[i] + m[i, cols]
            src = x[rows, cols] if x.dim() == 3 else x[rows]
            out[i, cols] = src.reshape(cols.numel(), K).to(x.dtype)
            wt[i, cols] = 1.0
    if negative_indices is not None:
        neg = T(negative_indices).reshape(-1).long()
        noff = _offsets(negative_indices, neg.shape[0])
        for i in range(N):
            cols = neg[noff[i]:noff[i + 1]]
            out[i, cols] = mv
            wt[i, cols] = 1.0
    return W(out), W(wt)


# ----------------------------------------------------------------------------- NMS
def _nms(boxes, scores, thr, eta=1.0, top_k=-1, normalized=True):
    order = torch.argsort(scores, descending=True, stable=True)
    if top_k > -1:
        order = order[:top_k]
    keep = []
    t = thr
    iou = _iou(boxes, boxes, normalized)
    for i in order.tolist():
        if all(float(iou[i, j]) <= t for j in keep):
            keep.append(i)
            if eta < 1.0 and t > 0.5:
                t *= eta
    return keep


def _multiclass(bb, sc, score_threshold, nms_top_k, keep_top_k, nms_threshold, normalized, nms_eta, background,
                merge=False):
    """one image: bb [M, 4] (or [M, C, 4]), sc [C, M] -> list of (label, score, box, index)"""
    dets = []
    for c in range(sc.shape[0]):
        if c == background:
            continue
        s = sc[c]
        cand = torch.nonzero(s > score_threshold).reshape(-1)
        if cand.numel() == 0:
            continue
        b = bb[:, c] if bb.dim() == 3 else bb
        boxes, ss = b[cand], s[cand]
        if merge:
            boxes, ss, cand = _locality_merge(boxes, ss, cand, nms_threshold, normalized)
        keep = _nms(boxes, ss, nms_threshold, nms_eta, nms_top_k, normalized)
        for k in keep:
            dets.append((c, float(ss[k]), boxes[k], int(cand[k])))
    dets.sort(key=lambda d: -d[1])
    if keep_top_k > -1:
        dets = dets[:keep_top_k]
    return dets


def _locality_merge(boxes, scores, idx, thr, normalized):
    """score-weighted merging of consecutive overlapping boxes (locality_aware_nms_op.cc)"""
    mb, ms, mi = [], [], []
    for k in range(boxes.shape[0]):
        if mb and float(_iou(mb[-1][None], boxes[k][None], normalized)[0, 0]) > thr:
            w0, w1 = ms[-1], float(scores[k])
            mb[-1] = (mb[-1] * w0 + boxes[k] * w1) / (w0 + w1)
            ms[-1] = w0 + w1
        else:
            mb.append(boxes[k].clone())
            ms.append(float(scores[k]))
            mi.append(int(idx[k]))
    return torch.stack(mb), torch.tensor(ms, device=boxes.device), torch.tensor(mi, device=boxes.device)


def _nms_output(all_dets, device, return_index=False, counts_only=False):
    rows, idx, lens = [], [], []
    for n, dets in enumerate(all_dets):
        for c, s, b, i in dets:
            rows.append(torch.cat([torch.tensor([float(c), s], device=device), b.float()]))
            idx.append(i)
        lens.append(len(dets))
    if not rows:
        out = _lod_out(torch.full((1, 1), -1.0, device=device), [1])
    else:
        out = _lod_out(torch.stack(rows), lens)
    if return_index:
        return out, W(torch.tensor(idx or [-1], dtype=torch.int64, device=device)[:, None])
    return out


def multiclass_nms(bboxes, scores, score_threshold, nms_top_k, keep_top_k, nms_threshold=0.3, normalized=True,
                   nms_eta=1.0, background_label=0, name=None):
    """bboxes [N, M, 4], scores [N, C, M] -> LoD [K, 6] rows (label, score, x1, y1, x2, y2); a
    single -1 row when nothing survives (multiclass_nms_op.cc)"""
    bb, sc = T(bboxes).float(), T(scores).float()
    dets = [_multiclass(bb[n], sc[n], score_threshold, nms_top_k, keep_top_k, nms_threshold, normalized, nms_eta,
                        background_label) for n in range(bb.shape[0])]
    return _nms_output(dets, bb.device)


def locality_aware_nms(bboxes, scores, score_threshold, nms_top_k, keep_top_k, nms_threshold=0.3, normalized=True,
                       nms_eta=1.0, background_label=-1, name=None):
    bb, sc = T(bboxes).float(), T(scores).float()
    dets = [_multiclass(bb[n], sc[n], score_threshold, nms_top_k, keep_top_k, nms_threshold, normalized, nms_eta,
                        background_label, merge=True) for n in range(bb.shape[0])]
    return _nms_output(dets, bb.device)


def matrix_nms(bboxes, scores, score_threshold, post_threshold, nms_top_k, keep_top_k, use_gaussian=False,
               gaussian_sigma=2.0, background_label=0, normalized=True, return_index=False, name=None):
    r = V.matrix_nms(bboxes, scores, score_threshold, post_threshold, nms_top_k, keep_top_k, use_gaussian,
                     gaussian_sigma, background_label, normalized, return_index, True)
    out, nums = r[0], r[1]
    out._lod = [fcore._offsets_from_lengths(T(nums).tolist())]
    return (out, r[2]) if return_index else out


def box_coder(prior_box, prior_box_var, target_box, code_type="encode_center_size", box_normalized=True, name=None,
              axis=0):
    return V.box_coder(prior_box, prior_box_var, target_box, code_type, box_normalized, axis)


def detection_output(loc, scores, prior_box, prior_box_var, background_label=0, nms_threshold=0.3, nms_top_k=400,
                     keep_top_k=200, score_threshold=0.01, nms_eta=1.0, return_index=False):
    """SSD head: decode ``loc`` against the priors, softmax the class scores, multiclass NMS"""
    lc = T(loc).float()
    N, M, _ = lc.shape
    dec = torch.stack([T(V.box_coder(prior_box, prior_box_var, W(lc[n]), "decode_center_size", True, 0))
                       .reshape(M, 4) for n in range(N)])
    sc = torch.softmax(T(scores).float(), -1).transpose(1, 2)
    dets = [_multiclass(dec[n], sc[n], score_threshold, nms_top_k, keep_top_k, nms_threshold, True, nms_eta,
                        background_label) for n in range(N)]
    return _nms_output(dets, lc.device, return_index)


def box_clip(input, im_info, name=None):
    """clip boxes to [0, im_w / scale - 1] x [0, im_h / scale - 1] of their image"""
    b = T(input).float()
    info = T(im_info).float()
    off = _offsets(input, b.shape[0]) if b.dim() == 2 else None
    out = b.clone()
    if off is None:
        for n in range(b.shape[0]):
            hw = torch.round(info[n, :2] / info[n, 2])
            out[n, ..., 0::2] = b[n, ..., 0::2].clamp(0, float(hw[1]) - 1)
            out[n, ..., 1::2] = b[n, ..., 1::2].clamp(0, float(hw[0]) - 1)
        return W(out)
    for n in range(len(off) - 1):
        hw = torch.round(info[n, :2] / info[n, 2])
        s = builtins_slice(off[n], off[n + 1])
        out[s, 0::2] = b[s, 0::2].clamp(0, float(hw[1]) - 1)
        out[s, 1::2] = b[s, 1::2].clamp(0, float(hw[0]) - 1)
    return W(out, input)


import builtins as _b  # noqa: E402
builtins_slice = _b.slice


def polygon_box_transform(input, name=None):
    """geometry offsets -> absolute coordinates: even channels 4*w - x, odd 4*h - x"""
    x = T(input)
    N, C, H, Wd = x.shape
    ww = torch.arange(Wd, device=x.device, dtype=x.dtype)[None, None, None, :].expand(N, C, H, Wd)
    hh = torch.arange(H, device=x.device, dtype=x.dtype)[None, None, :, None].expand(N, C, H, Wd)
    even = (torch.arange(C, device=x.device) % 2 == 0)[None, :, None, None]
    return W(torch.where(even, 4 * ww - x, 4 * hh - x))


def yolov3_loss(x, gt_box, gt_label, anchors, anchor_mask, class_num, ignore_thresh, downsample_ratio, gt_score=None,
                use_label_smooth=True, name=None, scale_x_y=1.0):
    return V.yolo_loss(x, gt_box, gt_label, anchors, anchor_mask, class_num, ignore_thresh, downsample_ratio, gt_score,
                       use_label_smooth, name, scale_x_y)


def yolo_box(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox=True, name=None,
             scale_x_y=1.0, iou_aware=False, iou_aware_factor=0.5):
    return V.yolo_box(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox, name, scale_x_y,
                      iou_aware, iou_aware_factor)


def sigmoid_focal_loss(x, label, fg_num, gamma=2.0, alpha=0.25):
    """label [N, 1] in 0..C (0 background, -1 ignored); per-element loss scaled by alpha / fg_num
    (positives) or (1 - alpha) / fg_num (negatives) (sigmoid_focal_loss_op.h)"""
    t = T(x).float()
    g = T(label).reshape(-1, 1).long()
    C = t.shape[1]
    d = torch.arange(C, device=t.device)[None, :]
    c_pos = (g == d + 1).float()
    c_neg = ((g != -1) & (g != d + 1)).float()
    fg = max(int(T(fg_num).reshape(-1)[0].item()), 1)
    p = torch.sigmoid(t)
    term_pos = (1 - p).pow(gamma) * torch.log(p.clamp_min(torch.finfo(torch.float32).tiny))
    term_neg = p.pow(gamma) * (-t * (t >= 0) - torch.log1p(torch.exp(t - 2 * t * (t >= 0))))
    return W(-c_pos * term_pos * (alpha / fg) - c_neg * term_neg * ((1 - alpha) / fg))


# ----------------------------------------------------------------------------- SSD loss
def ssd_loss(location, confidence, gt_box, gt_label, prior_box, prior_box_var=None, background_label=0,
             overlap_threshold=0.5, neg_pos_ratio=3.0, neg_overlap=0.5, loc_loss_weight=1.0, conf_loss_weight=1.0,
             match_type="per_prediction", mining_type="max_negative", normalize=True, sample_size=None):
    """SSD multibox loss: bipartite + per-prediction matching, max-negative hard mining,
    smooth-L1 on encoded targets + softmax CE; -> [N, 1] (normalised by the matched count)"""
    loc, conf = T(location).float(), T(confidence).float()
    gb, gl = T(gt_box).float(), T(gt_label).reshape(-1).long()
    pb = T(prior_box).float()
    N, P, C = conf.shape
    off = _offsets(gt_box, gb.shape[0])
    losses, total_pos = [], 0.0
    for n in range(N):
        g = gb[off[n]:off[n + 1]]
        lab = gl[off[n]:off[n + 1]]
        if g.shape[0] == 0:
            m = np.full(P, -1)
        else:
            m, _ = _bipartite(_iou(g, pb).cpu().numpy(), match_type, overlap_threshold)
        mt = torch.from_numpy(m).to(loc.device)
        pos = mt >= 0
        tgt_lab = torch.full((P,), background_label, dtype=torch.long, device=loc.device)
        tgt_lab[pos] = lab[mt[pos]]
        ce = TF.cross_entropy(conf[n], tgt_lab, reduction="none")
        # max-negative mining among unmatched priors whose best overlap < neg_overlap
        best = _iou(g, pb).max(0).values if g.shape[0] else torch.zeros(P, device=loc.device)
        cand = (~pos) & (best < neg_overlap)
        n_neg = int(min(int(cand.sum()), int(neg_pos_ratio * int(pos.sum()))))
        neg = torch.zeros_like(pos)
        if n_neg > 0:
            sc = torch.where(cand, ce.detach(), torch.full_like(ce, -1e30))
            neg[torch.topk(sc, n_neg).indices] = True
        conf_loss = (ce * (pos | neg).float()).sum()
        loc_loss = torch.zeros((), device=loc.device)
        if pos.any():
            enc = T(V.box_coder(W(pb[pos]), prior_box_var if prior_box_var is None else
                                W(T(prior_box_var).float()[pos]), W(g[mt[pos]]), "encode_center_size"))
            enc = torch.diagonal(enc, dim1=0, dim2=1).T if enc.dim() == 3 else enc
            d = loc[n][pos] - enc
            a = d.abs()
            loc_loss = torch.where(a < 1, 0.5 * d * d, a - 0.5).sum()
        losses.append(conf_loss_weight * conf_loss + loc_loss_weight * loc_loss)
        total_pos += float(pos.sum())
    out = torch.stack(losses)[:, None]
    if normalize:
        out = out / max(total_pos, 1.0)
    return W(out)


# ----------------------------------------------------------------------------- RPN / RetinaNet targets
def _sample_anchor_labels(iou, pos_thr, neg_thr, batch, fg_frac, use_random, rng):
    A = iou.shape[1]
    lab = torch.full((A,), -1, dtype=torch.long)
    if iou.shape[0] == 0:
        lab[:] = 0
        return lab, torch.zeros(A, dtype=torch.long)
    amax, arg = iou.max(0)
    gmax = iou.max(1).values
    lab[amax < neg_thr] = 0
    # each gt's best anchors are positive
    best = ((iou == gmax[:, None]) & (gmax[:, None] > 0)).any(0)
    lab[best] = 1
    lab[amax >= pos_thr] = 1
    if batch > 0:
        fg = torch.nonzero(lab == 1).reshape(-1)
        nfg = int(batch * fg_frac)
        if fg.numel() > nfg:
            drop = fg[torch.from_numpy(rng.permutation(fg.numel())[:fg.numel() - nfg])] if use_random else fg[nfg:]
            lab[drop] = -1
        bg = torch.nonzero(lab == 0).reshape(-1)
        nbg = batch - int((lab == 1).sum())
        if bg.numel() > nbg:
            drop = bg[torch.from_numpy(rng.permutation(bg.numel())[:bg.numel() - nbg])] if use_random else bg[nbg:]
            lab[drop] = -1
    return lab, arg


def _encode(anchors, gt, var=None):
    aw = anchors[:, 2] - anchors[:, 0] + 1.0
    ah = anchors[:, 3] - anchors[:, 1] + 1.0
    ax = anchors[:, 0] + 0.5 * aw
    ay = anchors[:, 1] + 0.5 * ah
    gw = gt[:, 2] - gt[:, 0] + 1.0
    gh = gt[:, 3] - gt[:, 1] + 1.0
    gx = gt[:, 0] + 0.5 * gw
    gy = gt[:, 1] + 0.5 * gh
    d = torch.stack([(gx - ax) / aw, (gy - ay) / ah, torch.log(gw / aw), torch.log(gh / ah)], 1)
    return d / var if var is not None else d


def rpn_target_assign(bbox_pred, cls_logits, anchor_box, anchor_var, gt_boxes, is_crowd, im_info,
                      rpn_batch_size_per_im=256, rpn_straddle_thresh=0.0, rpn_fg_fraction=0.5,
                      rpn_positive_overlap=0.7, rpn_negative_overlap=0.3, use_random=True):
    """-> (predicted_scores, predicted_location, target_label, target_bbox, bbox_inside_weight)
    over the sampled anchors of every image (rpn_target_assign_op.cc)"""
    bp, cl = T(bbox_pred).float(), T(cls_logits).float()
    an = T(anchor_box).float().reshape(-1, 4).cpu()
    gb = T(gt_boxes).float().cpu()
    crowd = T(is_crowd).reshape(-1).cpu()
    info = T(im_info).float().cpu()
    off = _offsets(gt_boxes, gb.shape[0])
    N = bp.shape[0]
    rng = np.random.RandomState(0)
    sl, ll, tl, tb, iw = [], [], [], [], []
    for n in range(N):
        inside = torch.ones(an.shape[0], dtype=torch.bool)
        if rpn_straddle_thresh >= 0:
            h, w = float(info[n, 0]), float(info[n, 1])
            t = rpn_straddle_thresh
            inside = (an[:, 0] >= -t) & (an[:, 1] >= -t) & (an[:, 2] < w + t) & (an[:, 3] < h + t)
        ids = torch.nonzero(inside).reshape(-1)
        g = gb[off[n]:off[n + 1]]
        g = g[crowd[off[n]:off[n + 1]] == 0] if crowd.numel() else g
        iou = _iou(g, an[ids], False)
        lab, arg = _sample_anchor_labels(iou, rpn_positive_overlap, rpn_negative_overlap, rpn_batch_size_per_im,
                                         rpn_fg_fraction, use_random, rng)
        fg = ids[lab == 1]
        keep = ids[lab >= 0]
        sl.append(cl[n].reshape(-1, 1)[keep.to(cl.device)])
        tl.append(lab[lab >= 0][:, None])
        ll.append(bp[n].reshape(-1, 4)[fg.to(bp.device)])
        tb.append(_encode(an[fg], g[arg[lab == 1]]) if fg.numel() else torch.zeros(0, 4))
        iw.append(torch.ones(fg.numel(), 4))
    d = bp.device
    return (W(torch.cat(sl)), W(torch.cat(ll)), W(torch.cat(tl).to(d).int()), W(torch.cat(tb).to(d)),
            W(torch.cat(iw).to(d)))


def retinanet_target_assign(bbox_pred, cls_logits, anchor_box, anchor_var, gt_boxes, gt_labels, is_crowd, im_info,
                            num_classes=1, positive_overlap=0.5, negative_overlap=0.4):
    """-> (predict_scores, predict_location, target_label, target_bbox, bbox_inside_weight,
    fg_num): every anchor with IoU >= positive_overlap (or a gt's best) is foreground, < negative
    is background; no sampling"""
    bp, cl = T(bbox_pred).float(), T(cls_logits).float()
    an = T(anchor_box).float().reshape(-1, 4).cpu()
    gb = T(gt_boxes).float().cpu()
    gl = T(gt_labels).reshape(-1).cpu().long()
    off = _offsets(gt_boxes, gb.shape[0])
    N = bp.shape[0]
    sl, ll, tl, tb, iw, fgn = [], [], [], [], [], []
    rng = np.random.RandomState(0)
    for n in range(N):
        g = gb[off[n]:off[n + 1]]
        labs = gl[off[n]:off[n + 1]]
        iou = _iou(g, an, False)
        lab, arg = _sample_anchor_labels(iou, positive_overlap, negative_overlap, -1, 1.0, False, rng)
        keep = torch.nonzero(lab >= 0).reshape(-1)
        fg = torch.nonzero(lab == 1).reshape(-1)
        cls_t = torch.zeros(keep.numel(), dtype=torch.long)
        fgmask = lab[keep] == 1
        cls_t[fgmask] = labs[arg[keep[fgmask]]]
        sl.append(cl[n].reshape(-1, num_classes)[keep.to(cl.device)])
        tl.append(cls_t[:, None])
        ll.append(bp[n].reshape(-1, 4)[fg.to(bp.device)])
        tb.append(_encode(an[fg], g[arg[fg]]) if fg.numel() else torch.zeros(0, 4))
        iw.append(torch.ones(fg.numel(), 4))
        fgn.append(fg.numel())
    d = bp.device
    return (W(torch.cat(sl)), W(torch.cat(ll)), W(torch.cat(tl).to(d).int()), W(torch.cat(tb).to(d)),
            W(torch.cat(iw).to(d)), W(torch.tensor([builtins_sum(fgn)], dtype=torch.int32, device=d)))


builtins_sum = _b.sum


def generate_proposals(scores, bbox_deltas, im_info, anchors, variances, pre_nms_top_n=6000, post_nms_top_n=1000,
                       nms_thresh=0.5, min_size=0.1, eta=1.0, return_rois_num=False, name=None):
    r = V.generate_proposals(scores, bbox_deltas, W(T(im_info)[:, :2]), anchors, variances, pre_nms_top_n,
                             post_nms_top_n, nms_thresh, min_size, eta, True, True)
    rois, probs, nums = r
    lens = T(nums).tolist()
    rois._lod = [fcore._offsets_from_lengths(lens)]
    probs._lod = [fcore._offsets_from_lengths(lens)]
    return (rois, probs, nums) if return_rois_num else (rois, probs)


def generate_proposal_labels(rpn_rois, gt_classes, is_crowd, gt_boxes, im_info, batch_size_per_im=256,
                             fg_fraction=0.25, fg_thresh=0.25, bg_thresh_hi=0.5, bg_thresh_lo=0.0,
                             bbox_reg_weights=[0.1, 0.1, 0.2, 0.2], class_nums=None, use_random=True,
                             is_cls_agnostic=False, is_cascade_rcnn=False, max_overlap=None,
                             return_max_overlap=False):
    """sample fg / bg RoIs (gt boxes appended) and build class-specific regression targets
    (generate_proposal_labels_op.cc) -> (rois, labels_int32, bbox_targets, bbox_inside_weights,
    bbox_outside_weights)"""
    rois = T(rpn_rois).float().cpu()
    gb = T(gt_boxes).float().cpu()
    gc = T(gt_classes).reshape(-1).long().cpu()
    info = T(im_info).float().cpu()
    roff = _offsets(rpn_rois, rois.shape[0])
    goff = _offsets(gt_boxes, gb.shape[0])
    K = class_nums or 2
    rng = np.random.RandomState(0)
    out_r, out_l, out_t, out_iw, lens = [], [], [], [], []
    wts = torch.tensor(bbox_reg_weights, dtype=torch.float32)
    for n in range(len(roff) - 1):
        scale = float(info[n, 2])
        g = gb[goff[n]:goff[n + 1]]
        r = torch.cat([rois[roff[n]:roff[n + 1]] / scale, g], 0)
        iou = _iou(r, g, False) if g.shape[0] else torch.zeros(r.shape[0], 1)
        mx, arg = iou.max(1)
        fg = torch.nonzero(mx >= fg_thresh).reshape(-1)
        bg = torch.nonzero((mx < bg_thresh_hi) & (mx >= bg_thresh_lo)).reshape(-1)
        nfg = min(int(batch_size_per_im * fg_fraction), fg.numel())
        if use_random and fg.numel() > nfg:
            fg = fg[torch.from_numpy(rng.permutation(fg.numel())[:nfg])]
        fg = fg[:nfg]
        nbg = min(batch_size_per_im - nfg, bg.numel())
        if use_random and bg.numel() > nbg:
            bg = bg[torch.from_numpy(rng.permutation(bg.numel())[:nbg])]
        bg = bg[:nbg]
        keep = torch.cat([fg, bg])
        lab = torch.zeros(keep.numel(), dtype=torch.long)
        lab[:fg.numel()] = gc[goff[n]:goff[n + 1]][arg[fg]] if g.shape[0] else 0
        sel = r[keep]
        tgt = torch.zeros(keep.numel(), 4 * K)
        iw = torch.zeros(keep.numel(), 4 * K)
        if fg.numel():
            d = _encode(sel[:fg.numel()], g[arg[fg]]) / wts
            for i in range(fg.numel()):
                c = 1 if is_cls_agnostic else int(lab[i])
                tgt[i, 4 * c:4 * c + 4] = d[i]
                iw[i, 4 * c:4 * c + 4] = 1.0
        out_r.append(sel * scale)
        out_l.append(lab[:, None])
        out_t.append(tgt)
        out_iw.append(iw)
        lens.append(keep.numel())
    d = dev()
    iw = torch.cat(out_iw).to(d)
    return (_lod_out(torch.cat(out_r).to(d), lens), _lod_out(torch.cat(out_l).to(d).int(), lens),
            _lod_out(torch.cat(out_t).to(d), lens), _lod_out(iw, lens), _lod_out(iw.clone(), lens))


def _poly_mask(polys, box, M):
    """rasterise polygons (lists of x, y) into an M x M grid over ``box`` (point-in-polygon at
    cell centres)"""
    x1, y1, x2, y2 = box
    w, h = max(x2 - x1, 1.0), max(y2 - y1, 1.0)
    ys, xs = np.meshgrid((np.arange(M) + 0.5) * h / M + y1, (np.arange(M) + 0.5) * w / M + x1, indexing="ij")
    mask = np.zeros((M, M), bool)
    for p in polys:
        px, py = np.asarray(p[0::2]), np.asarray(p[1::2])
        inside = np.zeros((M, M), bool)
        j = len(px) - 1
        for i in range(len(px)):
            cond = ((py[i] > ys) != (py[j] > ys)) & \
                (xs < (px[j] - px[i]) * (ys - py[i]) / (py[j] - py[i] + 1e-12) + px[i])
            inside ^= cond
            j = i
        mask |= inside
    return mask


def generate_mask_labels(im_info, gt_classes, is_crowd, gt_segms, rois, labels_int32, num_classes, resolution):
    """(mask_rois, roi_has_mask_int32, mask_int32 [R, num_classes * res^2]) for the foreground
    RoIs: the polygon of each RoI's best-overlapping gt, rasterised in the RoI
    (generate_mask_labels_op.cc). ``gt_segms`` is a 3-level LoD of polygon points."""
    info = T(im_info).float().cpu()
    r = T(rois).float().cpu()
    lab = T(labels_int32).reshape(-1).cpu()
    seg = T(gt_segms).float().cpu().reshape(-1, 2)
    slod = fcore.lod_of(gt_segms)          # [image -> gt, gt -> polygon, polygon -> point]
    roff = _offsets(rois, r.shape[0])
    out_r, out_h, out_m, lens = [], [], [], []
    for n in range(len(roff) - 1):
        scale = float(info[n, 2])
        gts = []
        for gi in range(slod[0][n], slod[0][n + 1]):
            polys = []
            for pi in range(slod[1][gi], slod[1][gi + 1]):
                pts = seg[slod[2][pi]:slod[2][pi + 1]]
                polys.append(pts.reshape(-1).tolist())
            gts.append(polys)
        boxes = torch.tensor([[min(p[0::2]), min(p[1::2]), max(p[0::2]), max(p[1::2])]
                              for polys in gts for p in polys[:1]] or [[0, 0, 0, 0]], dtype=torch.float32)
        rr = r[roff[n]:roff[n + 1]] / scale
        ll = lab[roff[n]:roff[n + 1]]
        fg = torch.nonzero(ll > 0).reshape(-1)
        masks = []
        for i in fg.tolist():
            best = int(_iou(rr[i:i + 1], boxes, False).argmax()) if gts else 0
            m = _poly_mask(gts[best], rr[i].tolist(), resolution) if gts else np.zeros((resolution,) * 2, bool)
            full = -np.ones((num_classes, resolution * resolution), np.int32)
            full[int(ll[i])] = m.reshape(-1).astype(np.int32)
            masks.append(full.reshape(-1))
        out_r.append(rr[fg] * scale)
        out_h.append(fg[:, None].int())
        out_m.append(torch.from_numpy(np.stack(masks)) if masks else
                     torch.zeros(0, num_classes * resolution * resolution, dtype=torch.int32))
        lens.append(fg.numel())
    d = dev()
    return (_lod_out(torch.cat(out_r).to(d), lens), _lod_out(torch.cat(out_h).to(d), lens),
            _lod_out(torch.cat(out_m).to(d), lens))


def roi_perspective_transform(input, rois, transformed_height, transformed_width, spatial_scale=1.0, name=None):
    """warp each quadrilateral RoI (x1, y1, ..., x4, y4) to a transformed_height x
    transformed_width patch by the perspective map of the output rectangle onto it, bilinear
    sampling -> (out, mask, transform_matrix) (roi_perspective_transform_op.cc)"""
    x = T(input).float()
    r = T(rois).float().cpu() * spatial_scale
    off = _offsets(rois, r.shape[0])
    bidx = []
    for n in range(len(off) - 1):
        bidx += [n] * (off[n + 1] - off[n])
    Ho, Wo = transformed_height, transformed_width
    outs, masks, mats = [], [], []
    for k in range(r.shape[0]):
        q = r[k].reshape(4, 2).double().numpy()
        src = np.array([[0, 0], [Wo - 1, 0], [Wo - 1, Ho - 1], [0, Ho - 1]], np.float64)
        A, bvec = [], []
        for (u, v), (X, Y) in zip(src, q):
            A.append([u, v, 1, 0, 0, 0, -u * X, -v * X])
            bvec.append(X)
            A.append([0, 0, 0, u, v, 1, -u * Y, -v * Y])
            bvec.append(Y)
        h = np.linalg.solve(np.array(A), np.array(bvec))
        Mx = np.append(h, 1.0).reshape(3, 3)
        mats.append(torch.from_numpy(Mx.reshape(-1)).float())
        vv, uu = np.meshgrid(np.arange(Ho), np.arange(Wo), indexing="ij")
        den = Mx[2, 0] * uu + Mx[2, 1] * vv + Mx[2, 2]
        px = (Mx[0, 0] * uu + Mx[0, 1] * vv + Mx[0, 2]) / den
        py = (Mx[1, 0] * uu + Mx[1, 1] * vv + Mx[1, 2]) / den
        H, Wd = x.shape[2:]
        inb = (px >= -0.5) & (px <= Wd - 0.5) & (py >= -0.5) & (py <= H - 0.5)
        gx = torch.from_numpy(px / max(Wd - 1, 1) * 2 - 1).float()
        gy = torch.from_numpy(py / max(H - 1, 1) * 2 - 1).float()
        grid = torch.stack([gx, gy], -1)[None].to(x.device)
        samp = TF.grid_sample(x[bidx[k]:bidx[k] + 1], grid, mode="bilinear", padding_mode="zeros",
                              align_corners=True)[0]
        m = torch.from_numpy(inb).to(x.device)
        outs.append(samp * m)
        masks.append(m.int()[None])
    return W(torch.stack(outs)), W(torch.stack(masks)), W(torch.stack(mats).to(x.device))


def retinanet_detection_output(bboxes, scores, anchors, im_info, score_threshold=0.05, nms_top_k=1000,
                               keep_top_k=100, nms_threshold=0.3, nms_eta=1.0):
    """per FPN level: top-k anchors over threshold, decode; then class-wise NMS over all levels"""
    info = T(im_info).float()
    N = T(bboxes[0]).shape[0]
    all_dets = []
    for n in range(N):
        boxes, scs = [], []
        for lb, ls, la in zip(bboxes, scores, anchors):
            d = T(lb)[n].float()
            s = T(ls)[n].float()
            a = T(la).float().reshape(-1, 4)
            flat = s.reshape(-1)
            cand = torch.nonzero(flat > score_threshold).reshape(-1)
            cand = cand[torch.argsort(flat[cand], descending=True)][:nms_top_k]
            ai = cand // s.shape[1]
            aw = a[ai, 2] - a[ai, 0] + 1
            ah = a[ai, 3] - a[ai, 1] + 1
            ax, ay = a[ai, 0] + 0.5 * aw, a[ai, 1] + 0.5 * ah
            dd = d[ai]
            cx, cy = dd[:, 0] * aw + ax, dd[:, 1] * ah + ay
            w, h = torch.exp(dd[:, 2]) * aw, torch.exp(dd[:, 3]) * ah
            b = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - 1, cy + h / 2 - 1], 1) / info[n, 2]
            b[:, 0::2] = b[:, 0::2].clamp(0, float(info[n, 1] / info[n, 2]) - 1)
            b[:, 1::2] = b[:, 1::2].clamp(0, float(info[n, 0] / info[n, 2]) - 1)
            sc = torch.full((s.shape[1], cand.numel()), -1.0, device=s.device)
            sc[cand % s.shape[1], torch.arange(cand.numel(), device=s.device)] = flat[cand]
            boxes.append(b)
            scs.append(sc)
        bb = torch.cat(boxes)
        ss = torch.cat(scs, 1)
        dets = _multiclass(bb, ss, score_threshold, -1, keep_top_k, nms_threshold, False, nms_eta, -1)
        all_dets.append([(c + 1, s, b, i) for c, s, b, i in dets])
    return _nms_output(all_dets, info.device)


def distribute_fpn_proposals(fpn_rois, min_level, max_level, refer_level, refer_scale, rois_num=None, name=None):
    return V.distribute_fpn_proposals(fpn_rois, min_level, max_level, refer_level, refer_scale, False, rois_num)


def box_decoder_and_assign(prior_box, prior_box_var, target_box, box_score, box_clip, name=None):
    """decode per-class deltas [R, 4C] against the priors; the assigned box is the decoded box of
    the best non-background class (box_decoder_and_assign_op.h)"""
    pb = T(prior_box).float()
    pv = T(prior_box_var).float().reshape(-1)
    tb = T(target_box).float()
    sc = T(box_score).float()
    R, C4 = tb.shape
    C = C4 // 4
    pw = pb[:, 2] - pb[:, 0] + 1
    ph = pb[:, 3] - pb[:, 1] + 1
    px, py = pb[:, 0] + pw / 2, pb[:, 1] + ph / 2
    d = tb.reshape(R, C, 4)
    dw = (pv[2] * d[..., 2]).clamp(max=box_clip)
    dh = (pv[3] * d[..., 3]).clamp(max=box_clip)
    cx = pv[0] * d[..., 0] * pw[:, None] + px[:, None]
    cy = pv[1] * d[..., 1] * ph[:, None] + py[:, None]
    w, h = torch.exp(dw) * pw[:, None], torch.exp(dh) * ph[:, None]
    dec = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - 1, cy + h / 2 - 1], -1)
    best = sc[:, 1:].argmax(1) + 1 if C > 1 else torch.zeros(R, dtype=torch.long, device=sc.device)
    assign = dec[torch.arange(R, device=dec.device), best]
    return W(dec.reshape(R, C4)), W(assign)


def collect_fpn_proposals(multi_rois, multi_scores, min_level, max_level, post_nms_top_n, rois_num_per_level=None,
                          name=None):
    """concatenate the RoIs of every level and keep each image's ``post_nms_top_n`` best"""
    L = max_level - min_level + 1
    rois = [T(r).float() for r in multi_rois[:L]]
    scs = [T(s).float().reshape(-1) for s in multi_scores[:L]]
    if rois_num_per_level is not None:
        nums = [T(n).reshape(-1).tolist() for n in rois_num_per_level[:L]]
    else:
        nums = [fcore._lengths_from_offsets(_offsets(r)) for r in multi_rois[:L]]
    N = len(nums[0])
    out, lens = [], []
    for n in range(N):
        rr, ss = [], []
        for lv in range(L):
            a = builtins_sum(nums[lv][:n])
            rr.append(rois[lv][a:a + nums[lv][n]])
            ss.append(scs[lv][a:a + nums[lv][n]])
        r, s = torch.cat(rr), torch.cat(ss)
        k = torch.argsort(s, descending=True, stable=True)[:post_nms_top_n]
        out.append(r[k])
        lens.append(k.numel())
    res = _lod_out(torch.cat(out), lens)
    if rois_num_per_level is not None:
        return res, W(torch.tensor(lens, dtype=torch.int32, device=dev()))
    return res


# every detection op records ONE op in a static Program (multi_box_head creates conv parameters:
# a builder); their data-dependent output rows (NMS keeps, proposals) come from static/program.py's
# example-run InferMeta as -1 dims
register(globals(), __all__, skip={"multi_box_head"})
