"""Detection ops (reference: python/paddle/vision/ops.py, phi/kernels/gpu/{roi_align,roi_pool,
psroi_pool,deformable_conv,yolo_box,nms}_kernel.cu). Implemented with batched tensor ops so
they run on the HIP device without per-box host loops (except NMS's sequential suppression,
done on a [N, N] IoU matrix)."""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as TF

from ..framework.core import Tensor, _wrap, default_device
from ..nn.layer.layers import Layer
from ..nn import initializer as I

__all__ = ["yolo_loss", "yolo_box", "deform_conv2d", "DeformConv2D", "distribute_fpn_proposals",
           "generate_proposals", "read_file", "decode_jpeg", "roi_pool", "RoIPool", "psroi_pool", "PSRoIPool",
           "roi_align", "RoIAlign", "nms", "box_coder", "prior_box", "matrix_nms"]


def _t(x):
    return None if x is None else (x._t if isinstance(x, Tensor) else torch.as_tensor(x))


def _box_iou(a, b):
    area_a = (a[:, 2] - a[:, 0]).clamp_min(0) * (a[:, 3] - a[:, 1]).clamp_min(0)
    area_b = (b[:, 2] - b[:, 0]).clamp_min(0) * (b[:, 3] - b[:, 1]).clamp_min(0)
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp_min(0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area_a[:, None] + area_b[None, :] - inter).clamp_min(1e-10)


def _nms_single(boxes, scores, thr):
    order = torch.argsort(scores, descending=True)
    b = boxes[order]
    iou = _box_iou(b, b).cpu().numpy()
    n = b.shape[0]
    keep = []
    removed = np.zeros(n, dtype=bool)
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        removed |= iou[i] > thr
    return order[torch.as_tensor(keep, dtype=torch.long, device=boxes.device)]


def nms(boxes, iou_threshold=0.3, scores=None, category_idxs=None, categories=None, top_k=None):
    bx = _t(boxes).float()
    sc = _t(scores).float() if scores is not None else torch.arange(bx.shape[0], 0, -1, device=bx.device).float()
    if category_idxs is None:
        keep = _nms_single(bx, sc, iou_threshold)
    else:
        cats = _t(category_idxs)
        keeps = []
        for c in (categories if categories is not None else torch.unique(cats).tolist()):
            idx = torch.nonzero(cats == c).reshape(-1)
            if idx.numel():
                keeps.append(idx[_nms_single(bx[idx], sc[idx], iou_threshold)])
        keep = torch.cat(keeps) if keeps else torch.zeros(0, dtype=torch.long, device=bx.device)
        keep = keep[torch.argsort(sc[keep], descending=True)]
    if top_k is not None:
        keep = keep[:top_k]
    return _wrap(keep)


def _roi_batch_index(boxes_num, n_rois, device):
    if boxes_num is None:
        return torch.zeros(n_rois, dtype=torch.long, device=device)
    bn = _t(boxes_num).long().to(device)
    return torch.repeat_interleave(torch.arange(bn.numel(), device=device), bn)


def roi_align(x, boxes, boxes_num, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=True, name=None):
    feat = _t(x)
    rois = _t(boxes).to(feat.dtype)
    N, C, H, W = feat.shape
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    bidx = _roi_batch_index(boxes_num, rois.shape[0], feat.device)
    off = 0.5 if aligned else 0.0
    x1, y1, x2, y2 = (rois[:, i] * spatial_scale - off for i in range(4))
    rw, rh = x2 - x1, y2 - y1
    if not aligned:
        rw, rh = rw.clamp_min(1.0), rh.clamp_min(1.0)
    sr = sampling_ratio if sampling_ratio > 0 else 2
    iy = (torch.arange(oh * sr, device=feat.device, dtype=feat.dtype) + 0.5) / sr
    ix = (torch.arange(ow * sr, device=feat.device, dtype=feat.dtype) + 0.5) / sr
    ys = y1[:, None] + iy[None, :] * (rh / oh)[:, None]
    xs = x1[:, None] + ix[None, :] * (rw / ow)[:, None]
    gy = ys / H * 2 - 1 + 1.0 / H
    gx = xs / W * 2 - 1 + 1.0 / W
    grid = torch.stack(torch.broadcast_tensors(gx[:, None, :], gy[:, :, None]), -1)
    samp = TF.grid_sample(feat[bidx], grid, mode="bilinear", padding_mode="zeros", align_corners=False)
    out = TF.avg_pool2d(samp, sr)
    return _wrap(out)


class RoIAlign(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num, aligned=True):
        return roi_align(x, boxes, boxes_num, self.output_size, self.spatial_scale, aligned=aligned)


def roi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    feat = _t(x)
    rois = _t(boxes)
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    bidx = _roi_batch_index(boxes_num, rois.shape[0], feat.device)
    outs = []
    for i in range(rois.shape[0]):
        x1, y1, x2, y2 = (int(round(float(v) * spatial_scale)) for v in rois[i])
        x2, y2 = max(x2, x1), max(y2, y1)
        crop = feat[bidx[i], :, y1:y2 + 1, x1:x2 + 1]
        outs.append(TF.adaptive_max_pool2d(crop, (oh, ow)))
    return _wrap(torch.stack(outs) if outs else feat.new_zeros(0, feat.shape[1], oh, ow))


class RoIPool(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return roi_pool(x, boxes, boxes_num, self.output_size, self.spatial_scale)


def psroi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    feat = _t(x)
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    pooled = _t(roi_align(_wrap(feat), boxes, boxes_num, (oh, ow), spatial_scale, 2, False))
    R, C = pooled.shape[:2]
    cout = C // (oh * ow)
    pooled = pooled.reshape(R, cout, oh, ow, oh, ow)
    idx = torch.arange(oh, device=feat.device)
    jdx = torch.arange(ow, device=feat.device)
    out = pooled[:, :, idx[:, None], jdx[None, :], idx[:, None], jdx[None, :]]
    return _wrap(out)


class PSRoIPool(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return psroi_pool(x, boxes, boxes_num, self.output_size, self.spatial_scale)


def deform_conv2d(x, offset, weight, bias=None, stride=1, padding=0, dilation=1, deformable_groups=1, groups=1,
                  mask=None, name=None):
    """Deformable conv v1/v2 via bilinear sampling of the k*k taps then a grouped 1x1 GEMM."""
    inp, off, w = _t(x), _t(offset), _t(weight)
    N, C, H, W = inp.shape
    Co, Cg, kh, kw = w.shape
    s = stride if isinstance(stride, (list, tuple)) else (stride, stride)
    p = padding if isinstance(padding, (list, tuple)) else (padding, padding)
    d = dilation if isinstance(dilation, (list, tuple)) else (dilation, dilation)
    Ho = (H + 2 * p[0] - (d[0] * (kh - 1) + 1)) // s[0] + 1
    Wo = (W + 2 * p[1] - (d[1] * (kw - 1) + 1)) // s[1] + 1
    dg = deformable_groups
    off = off.reshape(N, dg, kh * kw, 2, Ho, Wo)
    base_y = (torch.arange(Ho, device=inp.device) * s[0] - p[0]).view(1, Ho, 1)
    base_x = (torch.arange(Wo, device=inp.device) * s[1] - p[1]).view(1, 1, Wo)
    ky = (torch.arange(kh, device=inp.device) * d[0]).repeat_interleave(kw).view(kh * kw, 1, 1)
    kx = (torch.arange(kw, device=inp.device) * d[1]).repeat(kh).view(kh * kw, 1, 1)
    cols = []
    cpg = C // dg
    for g in range(dg):
        yy = base_y + ky + off[:, g, :, 0]
        xx = base_x + kx + off[:, g, :, 1]
        grid = torch.stack([xx / max(W - 1, 1) * 2 - 1, yy / max(H - 1, 1) * 2 - 1], -1)
        grid = grid.reshape(N, kh * kw * Ho, Wo, 2).to(inp.dtype)
        samp = TF.grid_sample(inp[:, g * cpg:(g + 1) * cpg], grid, mode="bilinear", padding_mode="zeros", align_corners=True)
        samp = samp.reshape(N, cpg, kh * kw, Ho, Wo)
        if mask is not None:
            m = _t(mask).reshape(N, dg, kh * kw, Ho, Wo)[:, g]
            samp = samp * m[:, None]
        cols.append(samp)
    col = torch.cat(cols, 1)                                  # [N, C, k, Ho, Wo]
    col = col.reshape(N, groups, C // groups * kh * kw, Ho * Wo)
    wg = w.reshape(groups, Co // groups, Cg * kh * kw)
    out = torch.einsum("gok,ngkl->ngol", wg, col).reshape(N, Co, Ho, Wo)
    if bias is not None:
        out = out + _t(bias).view(1, -1, 1, 1)
    return _wrap(out)


class DeformConv2D(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, deformable_groups=1,
                 groups=1, weight_attr=None, bias_attr=None):
        super().__init__()
        k = kernel_size if isinstance(kernel_size, (list, tuple)) else (kernel_size, kernel_size)
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._deformable_groups, self._groups = deformable_groups, groups
        fan_in = in_channels // groups * k[0] * k[1]
        self.weight = self.create_parameter([out_channels, in_channels // groups, k[0], k[1]], attr=weight_attr,
                                            default_initializer=I.Normal(0.0, (2.0 / fan_in) ** 0.5))
        self.bias = self.create_parameter([out_channels], attr=bias_attr, is_bias=True)

    def forward(self, x, offset, mask=None):
        return deform_conv2d(x, offset, self.weight, self.bias, self._stride, self._padding, self._dilation,
                             self._deformable_groups, self._groups, mask)


def yolo_box(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox=True, name=None,
             scale_x_y=1.0, iou_aware=False, iou_aware_factor=0.5):
    t = _t(x).float()
    N, _, H, W = t.shape
    na = len(anchors) // 2
    ioup = None
    if iou_aware:   # the first na channels are the IoU predictions (reference yolo_box kernel)
        ioup, t = t[:, :na], t[:, na:]
    t = t.reshape(N, na, 5 + class_num, H, W)
    img = _t(img_size).float()
    gy, gx = torch.meshgrid(torch.arange(H, device=t.device), torch.arange(W, device=t.device), indexing="ij")
    an = torch.tensor(anchors, dtype=torch.float32, device=t.device).reshape(na, 2)
    bias = -0.5 * (scale_x_y - 1)
    cx = (gx + torch.sigmoid(t[:, :, 0]) * scale_x_y + bias) / W
    cy = (gy + torch.sigmoid(t[:, :, 1]) * scale_x_y + bias) / H
    bw = torch.exp(t[:, :, 2]) * an[None, :, 0, None, None] / (downsample_ratio * W)
    bh = torch.exp(t[:, :, 3]) * an[None, :, 1, None, None] / (downsample_ratio * H)
    imh, imw = img[:, 0].view(N, 1, 1, 1), img[:, 1].view(N, 1, 1, 1)
    x1, y1 = (cx - bw / 2) * imw, (cy - bh / 2) * imh
    x2, y2 = (cx + bw / 2) * imw, (cy + bh / 2) * imh
    if clip_bbox:
        x1, y1 = x1.clamp(min=0), y1.clamp(min=0)
        x2, y2 = torch.minimum(x2, imw - 1), torch.minimum(y2, imh - 1)
    conf = torch.sigmoid(t[:, :, 4])
    if ioup is not None:
        conf = conf ** (1.0 - iou_aware_factor) * torch.sigmoid(ioup) ** iou_aware_factor
    probs = torch.sigmoid(t[:, :, 5:]) * conf[:, :, None]
    keep = (conf >= conf_thresh).float()
    boxes = torch.stack([x1, y1, x2, y2], -1) * keep[..., None]
    boxes = boxes.reshape(N, -1, 4)
    scores = (probs * keep[:, :, None]).permute(0, 1, 3, 4, 2).reshape(N, -1, class_num)
    return _wrap(boxes), _wrap(scores)


def yolo_loss(x, gt_box, gt_label, anchors, anchor_mask, class_num, ignore_thresh, downsample_ratio, gt_score=None,
              use_label_smooth=True, name=None, scale_x_y=1.0):
    """YOLOv3 loss (reference: phi/kernels/cpu/yolo_loss_kernel.cc) — box/objectness/class terms per image."""
    t = _t(x).float()
    N, _, H, W = t.shape
    mask = list(anchor_mask)
    na = len(mask)
    t = t.reshape(N, na, 5 + class_num, H, W)
    an = torch.tensor(anchors, dtype=torch.float32, device=t.device).reshape(-1, 2)
    gb = _t(gt_box).float()
    gl = _t(gt_label).long()
    gs = _t(gt_score).float() if gt_score is not None else torch.ones(gl.shape, device=t.device)
    input_size = downsample_ratio * H
    loss = torch.zeros(N, device=t.device)
    obj_target = torch.zeros(N, na, H, W, device=t.device)
    obj_weight = torch.ones(N, na, H, W, device=t.device)
    # ignore mask: predicted boxes overlapping any gt above threshold
    gy, gx = torch.meshgrid(torch.arange(H, device=t.device), torch.arange(W, device=t.device), indexing="ij")
    pcx = (gx + torch.sigmoid(t[:, :, 0])) / W
    pcy = (gy + torch.sigmoid(t[:, :, 1])) / H
    pw = torch.exp(t[:, :, 2]) * an[mask][None, :, 0, None, None] / input_size
    ph = torch.exp(t[:, :, 3]) * an[mask][None, :, 1, None, None] / input_size
    pbox = torch.stack([pcx - pw / 2, pcy - ph / 2, pcx + pw / 2, pcy + ph / 2], -1)
    for n in range(N):
        valid = (gb[n, :, 2] > 0) & (gb[n, :, 3] > 0)
        g = gb[n][valid]
        if g.numel():
            gxyxy = torch.stack([g[:, 0] - g[:, 2] / 2, g[:, 1] - g[:, 3] / 2, g[:, 0] + g[:, 2] / 2, g[:, 1] + g[:, 3] / 2], -1)
            iou = _box_iou(pbox[n].reshape(-1, 4), gxyxy).max(-1).values.reshape(na, H, W)
            obj_weight[n] = (iou <= ignore_thresh).float()
        for j in torch.nonzero(valid).reshape(-1).tolist():
            bx, by, bw, bh = gb[n, j].tolist()
            wh = torch.tensor([bw, bh], device=t.device) * input_size
            inter = torch.minimum(an[:, 0], wh[0]) * torch.minimum(an[:, 1], wh[1])
            iou_a = inter / (an[:, 0] * an[:, 1] + wh[0] * wh[1] - inter)
            best = int(torch.argmax(iou_a))
            if best not in mask:
                continue
            k = mask.index(best)
            gi, gj = int(bx * W), int(by * H)
            gi, gj = min(max(gi, 0), W - 1), min(max(gj, 0), H - 1)
            tx, ty = bx * W - gi, by * H - gj
            tw = math.log(max(bw * input_size / float(an[best, 0]), 1e-9))
            th = math.log(max(bh * input_size / float(an[best, 1]), 1e-9))
            sc = (2.0 - bw * bh) * float(gs[n, j])
            p = t[n, k, :, gj, gi]
            loss[n] = loss[n] + sc * (TF.binary_cross_entropy_with_logits(p[0], torch.tensor(tx, device=t.device)) +
                                      TF.binary_cross_entropy_with_logits(p[1], torch.tensor(ty, device=t.device)) +
                                      torch.abs(p[2] - tw) + torch.abs(p[3] - th))
            lab = torch.full((class_num,), 1.0 / class_num if use_label_smooth else 0.0, device=t.device)
            pos = 1.0 - 1.0 / class_num if use_label_smooth else 1.0
            lab[int(gl[n, j])] = pos
            loss[n] = loss[n] + float(gs[n, j]) * TF.binary_cross_entropy_with_logits(p[5:], lab, reduction="sum")
            obj_target[n, k, gj, gi] = float(gs[n, j])
            obj_weight[n, k, gj, gi] = 1.0
    obj = TF.binary_cross_entropy_with_logits(t[:, :, 4], obj_target, reduction="none") * obj_weight
    loss = loss + obj.reshape(N, -1).sum(-1)
    return _wrap(loss)


def distribute_fpn_proposals(fpn_rois, min_level, max_level, refer_level, refer_scale, pixel_offset=False,
                             rois_num=None, name=None):
    rois = _t(fpn_rois).float()
    off = 1.0 if pixel_offset else 0.0
    w = rois[:, 2] - rois[:, 0] + off
    h = rois[:, 3] - rois[:, 1] + off
    lvl = torch.floor(torch.log2(torch.sqrt(w * h).clamp_min(1e-6) / refer_scale + 1e-8) + refer_level)
    lvl = lvl.clamp(min_level, max_level).long()
    multi, restore = [], []
    order = []
    for l in range(min_level, max_level + 1):
        idx = torch.nonzero(lvl == l).reshape(-1)
        multi.append(_wrap(rois[idx]))
        order.append(idx)
    cat = torch.cat(order)
    restore_ind = torch.empty_like(cat)
    restore_ind[cat] = torch.arange(cat.numel(), device=cat.device)
    nums = None
    if rois_num is not None:
        nums = [_wrap(torch.tensor([m._t.shape[0]], dtype=torch.int32)) for m in multi]
    return multi, _wrap(restore_ind.reshape(-1, 1)), nums


def box_coder(prior_box, prior_box_var, target_box, code_type="encode_center_size", box_normalized=True, axis=0, name=None):
    pb, tb = _t(prior_box).float(), _t(target_box).float()
    pv = _t(prior_box_var).float() if isinstance(prior_box_var, (Tensor, torch.Tensor, np.ndarray)) else \
        torch.tensor(prior_box_var if prior_box_var is not None else [1.0, 1.0, 1.0, 1.0], device=pb.device)
    """reference phi box_coder kernel (oracle: test_box_coder_op.py box_encoder / box_decoder):
    prior centres include the +1 of unnormalized boxes, encoded target centres are plain
    midpoints; ``axis`` says which dimension of a decode input the M priors run along"""
    code_type = code_type.lower()
    off = 0.0 if box_normalized else 1.0
    pw = pb[:, 2] - pb[:, 0] + off
    ph = pb[:, 3] - pb[:, 1] + off
    pcx = pb[:, 0] + pw / 2
    pcy = pb[:, 1] + ph / 2
    if code_type in ("encode_center_size", "encodecentersize"):
        tw = tb[:, 2] - tb[:, 0] + off
        th = tb[:, 3] - tb[:, 1] + off
        tcx = (tb[:, 0] + tb[:, 2]) / 2
        tcy = (tb[:, 1] + tb[:, 3]) / 2
        out = torch.stack([(tcx[:, None] - pcx) / pw, (tcy[:, None] - pcy) / ph,
                           torch.log(torch.abs(tw[:, None] / pw)), torch.log(torch.abs(th[:, None] / ph))], -1)
        return _wrap(out / pv.reshape(1, -1, 4) if pv.dim() > 1 else out / pv)
    shp = (1, -1) if axis == 0 else (-1, 1)
    pw, ph, pcx, pcy = pw.reshape(shp), ph.reshape(shp), pcx.reshape(shp), pcy.reshape(shp)
    v = pv.reshape(shp + (4,)) if pv.dim() > 1 else pv.view(1, 1, 4)
    d = tb if tb.dim() == 3 else tb.unsqueeze(1)
    cx = v[..., 0] * d[..., 0] * pw + pcx
    cy = v[..., 1] * d[..., 1] * ph + pcy
    w = torch.exp(v[..., 2] * d[..., 2]) * pw
    h = torch.exp(v[..., 3] * d[..., 3]) * ph
    return _wrap(torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - off, cy + h / 2 - off], -1))


def prior_box(input, image, min_sizes, max_sizes=None, aspect_ratios=[1.0], variance=[0.1, 0.1, 0.2, 0.2], flip=False,
              clip=False, steps=[0.0, 0.0], offset=0.5, min_max_aspect_ratios_order=False, name=None):
    H, W = _t(input).shape[2:]
    IH, IW = _t(image).shape[2:]
    sw = steps[0] or IW / W
    sh = steps[1] or IH / H
    ars = [1.0]
    for a in aspect_ratios:
        if all(abs(a - x) > 1e-6 for x in ars):
            ars.append(a)
            if flip:
                ars.append(1.0 / a)
    boxes = []
    for i in range(H):
        for j in range(W):
            cx, cy = (j + offset) * sw, (i + offset) * sh
            for k, ms in enumerate(min_sizes):
                cell = []
                for a in ars:
                    bw, bh = ms * math.sqrt(a) / 2, ms / math.sqrt(a) / 2
                    cell.append([(cx - bw) / IW, (cy - bh) / IH, (cx + bw) / IW, (cy + bh) / IH])
                if max_sizes:
                    # reference prior_box kernel: [ar = 1, max, other ars] when
                    # min_max_aspect_ratios_order, else [every ar, max]
                    s = math.sqrt(ms * max_sizes[k]) / 2
                    mx = [(cx - s) / IW, (cy - s) / IH, (cx + s) / IW, (cy + s) / IH]
                    if min_max_aspect_ratios_order:
                        cell.insert(1, mx)
                    else:
                        cell.append(mx)
                boxes.extend(cell)
    b = torch.tensor(boxes, dtype=torch.float32, device=default_device()).reshape(H, W, -1, 4)
    if clip:
        b = b.clamp(0, 1)
    v = torch.tensor(variance, dtype=torch.float32, device=b.device).expand_as(b)
    return _wrap(b), _wrap(v.contiguous())


def generate_proposals(scores, bbox_deltas, img_size, anchors, variances, pre_nms_top_n=6000, post_nms_top_n=1000,
                       nms_thresh=0.5, min_size=0.1, eta=1.0, pixel_offset=False, return_rois_num=False, name=None):
    sc, dl, an, var = _t(scores).float(), _t(bbox_deltas).float(), _t(anchors).float(), _t(variances).float()
    im = _t(img_size).float()
    N = sc.shape[0]
    an = an.reshape(-1, 4)
    var = var.reshape(-1, 4)
    rois, probs, nums = [], [], []
    for n in range(N):
        s = sc[n].permute(1, 2, 0).reshape(-1)
        d = dl[n].permute(1, 2, 0).reshape(-1, 4)
        k = min(pre_nms_top_n, s.numel())
        top = torch.topk(s, k).indices
        boxes = _t(box_coder(_wrap(an[top]), _wrap(var[top]), _wrap(d[top].unsqueeze(1)), "decode_center_size",
                             not pixel_offset)).reshape(-1, 4)
        boxes[:, 0::2] = boxes[:, 0::2].clamp(0, float(im[n, 1]) - 1)
        boxes[:, 1::2] = boxes[:, 1::2].clamp(0, float(im[n, 0]) - 1)
        keep = ((boxes[:, 2] - boxes[:, 0]) >= min_size) & ((boxes[:, 3] - boxes[:, 1]) >= min_size)
        boxes, ss = boxes[keep], s[top][keep]
        kk = _nms_single(boxes, ss, nms_thresh)[:post_nms_top_n]
        rois.append(boxes[kk])
        probs.append(ss[kk].unsqueeze(-1))
        nums.append(kk.numel())
    out = (_wrap(torch.cat(rois)), _wrap(torch.cat(probs)))
    if return_rois_num:
        out = out + (_wrap(torch.tensor(nums, dtype=torch.int32)),)
    return out


def matrix_nms(bboxes, scores, score_threshold, post_threshold, nms_top_k, keep_top_k, use_gaussian=False,
               gaussian_sigma=2.0, background_label=0, normalized=True, return_index=False, return_rois_num=True, name=None):
    bb, sc = _t(bboxes).float(), _t(scores).float()
    outs, idxs, nums = [], [], []
    for n in range(bb.shape[0]):
        dets = []
        for c in range(sc.shape[1]):
            if c == background_label:
                continue
            s = sc[n, c]
            cand = torch.nonzero(s > score_threshold).reshape(-1)
            if cand.numel() == 0:
                continue
            cand = cand[torch.argsort(s[cand], descending=True)][:nms_top_k]
            b = bb[n, cand]
            iou = torch.triu(_box_iou(b, b), 1)
            comp = iou.max(0).values
            decay = torch.exp(-(iou ** 2 - comp[:, None] ** 2) / gaussian_sigma) if use_gaussian else (1 - iou) / (1 - comp[:, None])
            dec = decay.min(0).values
            ns = s[cand] * dec
            keep = ns > post_threshold
            for i in torch.nonzero(keep).reshape(-1).tolist():
                dets.append((float(ns[i]), c, b[i], int(cand[i])))
        dets.sort(key=lambda d: -d[0])
        dets = dets[:keep_top_k]
        for s_, c_, b_, i_ in dets:
            outs.append(torch.cat([torch.tensor([c_, s_], device=bb.device), b_]))
            idxs.append(i_)
        nums.append(len(dets))
    out = _wrap(torch.stack(outs) if outs else torch.zeros(0, 6, device=bb.device))
    res = [out]
    if return_rois_num:
        res.append(_wrap(torch.tensor(nums, dtype=torch.int32)))
    if return_index:
        res.append(_wrap(torch.tensor(idxs, dtype=torch.int64)))
    return tuple(res) if len(res) > 1 else out


def read_file(filename, name=None):
    with open(filename, "rb") as f:
        data = np.frombuffer(f.read(), dtype=np.uint8)
    return _wrap(torch.from_numpy(data.copy()))


def decode_jpeg(x, mode="unchanged", name=None):
    import io
    from PIL import Image
    buf = bytes(_t(x).cpu().numpy().tobytes())
    img = Image.open(io.BytesIO(buf))
    if mode == "gray":
        img = img.convert("L")
    elif mode == "rgb":
        img = img.convert("RGB")
    arr = np.asarray(img)
    if arr.ndim == 2:
        arr = arr[None]
    else:
        arr = arr.transpose(2, 0, 1)
    return _wrap(torch.from_numpy(arr.copy()).to(default_device()))
