"""Per-convolution efficiency table of one ResNet-50 training step (NHWC, bf16, batch 256 by default):
every call into the own conv kernels (``conv256_fwd`` — forward and dgrad phases — and
``conv256_wgrad``) is recorded during one step, then each distinct call is replayed alone and timed
with events. Prints TF/s and the effective HBM traffic (operands read once + output written once)
against the two rooflines, so the time lost per shape is visible:

    python tools/resnet_conv_table.py [batch]

``bound`` = max(flops / 2.3 PF/s, bytes / 5.3 TB/s) — the better of the sustained MFMA and copy
ceilings measured on this box (profiles/hbm_ceilings_r5.log, profiles/tn_wgrad_r5/)."""
import os
import sys
from collections import OrderedDict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_hackathon_amd as paddle  # noqa: E402
from paddle_hackathon_amd.ops import conv_gemm  # noqa: E402
from paddle_hackathon_amd.vision.models import resnet50  # noqa: E402

PEAK_F, PEAK_B = 2.3e15, 5.3e12


def _fwd_geo(x, w, stride, padding, dilation, remap):
    N, H, W, C = x.shape
    Co, KH, KW, _ = w.shape
    if remap is not None:
        OH, OW = remap[4], remap[5]
    else:
        OH = (H + 2 * padding[0] - dilation[0] * (KH - 1) - 1) // stride[0] + 1
        OW = (W + 2 * padding[1] - dilation[1] * (KW - 1) - 1) // stride[1] + 1
    fl = 2.0 * N * OH * OW * Co * KH * KW * C
    by = 2.0 * (x.numel() + w.numel() + N * OH * OW * Co)
    return fl, by, f"{N}x{H}x{W}x{C}->{Co} k{KH}x{KW} s{stride[0]} out {OH}x{OW}"


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    paddle.set_device("gpu")
    paddle.seed(0)
    model = paddle.amp.decorate(resnet50(data_format="NHWC"), level="O2", dtype="bfloat16")
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=model.parameters(),
                                    multi_precision=True)
    x = paddle.to_tensor(torch.randn(B, 224, 224, 3, device="cuda").bfloat16())
    y = paddle.to_tensor(torch.randint(0, 1000, (B,), device="cuda"))

    def step():
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            loss = paddle.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)

    for _ in range(2):
        step()
    torch.cuda.synchronize()

    rec = []
    of, ow = conv_gemm.conv256_fwd, conv_gemm.conv256_wgrad

    def fwd(*a, **kw):
        rec.append(("fwd", a, kw))
        return of(*a, **kw)

    def wgr(*a, **kw):
        rec.append(("wgrad", a, kw))
        return ow(*a, **kw)
    conv_gemm.conv256_fwd, conv_gemm.conv256_wgrad = fwd, wgr
    # whole-step event time for the share column
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    step()
    e.record()
    torch.cuda.synchronize()
    step_ms = s.elapsed_time(e)
    conv_gemm.conv256_fwd, conv_gemm.conv256_wgrad = of, ow

    rows = OrderedDict()
    for kind, a, kw in rec:
        if kind == "fwd":
            xx, w, stride, padding, dilation = a[:5]
            remap = kw.get("remap")
            tag = "dgrad" if remap is not None else "fwd"
            fl, by, desc = _fwd_geo(xx, w, stride, padding, dilation, remap)
            if kw.get("addend") is not None:
                by += 2.0 * kw["addend"].numel()
            fn = (lambda a=a, kw=kw: of(*a, **kw))
        else:
            dy, xx, w_shape, stride, padding, dilation = a[:6]
            Co, Ci, KH, KW = w_shape
            N, OH, OW, _ = dy.shape
            fl = 2.0 * N * OH * OW * Co * KH * KW * Ci
            by = 2.0 * (dy.numel() + xx.numel() + Co * Ci * KH * KW)
            desc = f"{tuple(xx.shape)} dy {OH}x{OW}x{Co} k{KH}x{KW} s{stride[0]}"
            tag = "wgrad"
            fn = (lambda a=a, kw=kw: ow(*a, **kw))
        key = (tag, desc)
        if key not in rows:
            rows[key] = [0, fl, by, fn]
        rows[key][0] += 1

    tot = tot_bound = 0.0
    out = []
    for (tag, desc), (n, fl, by, fn) in rows.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        it = 20
        s.record()
        for _ in range(it):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / it
        bound = max(fl / PEAK_F, by / PEAK_B) * 1e3
        tot += ms * n
        tot_bound += bound * n
        out.append((ms * n, tag, desc, n, ms, fl / ms / 1e9, by / ms / 1e6, bound))
    out.sort(reverse=True)
    print(f"ResNet-50 NHWC bf16 batch {B}: step {step_ms:.2f} ms (event, eager), {len(rec)} conv kernel calls, "
          f"{len(rows)} distinct")
    print(f"conv total (isolated replays) {tot:.2f} ms/step, roofline bound {tot_bound:.2f} ms "
          f"({100 * tot_bound / tot:.0f} % of SOL)")
    print(f"{'ms/step':>8} {'kind':5} {'n':>2} {'us/call':>8} {'TF/s':>6} {'GB/s':>6} {'SOL us':>7} {'%SOL':>5}  shape")
    for tms, tag, desc, n, ms, tf, gbs, bound in out:
        print(f"{tms:8.3f} {tag:5} {n:2d} {ms * 1e3:8.1f} {tf:6.0f} {gbs:6.0f} {bound * 1e3:7.1f} "
              f"{100 * bound / ms:5.0f}  {desc}")


if __name__ == "__main__":
    main()
