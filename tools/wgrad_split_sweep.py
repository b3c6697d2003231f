"""Tile x split-K sweep of the conv weight-gradient kernel (pha_conv256_wgrad) on the ResNet-50
training shapes (batch 256, NHWC bf16): for each shape, the time of the current choice (table tile,
formula splits, as conv_gemm.conv256_wgrad runs it) against every candidate tile with split factors
1..512, so a better split policy is visible per shape.

    python tools/wgrad_split_sweep.py [batch]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_hackathon_amd.ops import conv_gemm as cg  # noqa: E402

# (H, W, Ci, Co, k, stride, pad) of the ResNet-50 convolutions (input spatial size)
SHAPES = [
    (56, 56, 64, 64, 3, 1, 1), (28, 28, 128, 128, 3, 1, 1), (14, 14, 256, 256, 3, 1, 1), (7, 7, 512, 512, 3, 1, 1),
    (56, 56, 128, 128, 3, 2, 1), (28, 28, 256, 256, 3, 2, 1), (14, 14, 512, 512, 3, 2, 1),
    (56, 56, 64, 256, 1, 1, 0), (56, 56, 256, 64, 1, 1, 0), (28, 28, 128, 512, 1, 1, 0), (28, 28, 512, 128, 1, 1, 0),
    (14, 14, 256, 1024, 1, 1, 0), (14, 14, 1024, 256, 1, 1, 0), (7, 7, 512, 2048, 1, 1, 0), (7, 7, 2048, 512, 1, 1, 0),
    (224, 224, 8, 64, 7, 2, 3),
]


def _time(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda")
    L, z = cg._L256(), cg._ptr(cg._zero_page(dev))
    from ctypes import c_void_p
    st = c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    tot_cur = tot_best = 0.0
    for (H, W, Ci, Co, k, s, p) in SHAPES:
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(B, H, W, Ci, device=dev).bfloat16()
        dy = torch.randn(B, OH, OW, Co, device=dev).bfloat16()
        out = torch.empty(Co, Ci, k, k, dtype=torch.bfloat16, device=dev)
        M, N, K = Co, k * k * Ci, B * OH * OW
        fl = 2.0 * M * N * K

        def call(tile, sp, ws):
            rc = L.pha_conv256_wgrad(cg._DT[dy.dtype], cg._ptr(dy), cg._ptr(x), cg._ptr(out), cg._ptr(ws), B, H, W,
                                     Ci, Co, k, k, s, s, p, p, 1, 1, 0, z, tile, sp, st)
            assert rc == 0, rc
        ref = cg.conv256_wgrad(dy, x, (Co, Ci, k, k), (s, s), (p, p), (1, 1)).float()
        cur = _time(lambda: cg.conv256_wgrad(dy, x, (Co, Ci, k, k), (s, s), (p, p), (1, 1)))
        best = (cur, None, None)
        line = []
        for t in cg._tn_tiles(M, N):
            kb = -(-K // 32)
            for sp in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512):
                if sp > kb // 4:
                    break
                ws = cg._tn_ws(sp, M, N, dev)
                us = _time(lambda: call(t, sp, ws))
                if us < best[0]:
                    call(t, sp, ws)
                    err = (out.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
                    assert err < 2e-2, (t, sp, err)
                    best = (us, t, sp)
            line.append(t)
        tot_cur += cur
        tot_best += best[0]
        bt = cg._TN_CANDS[best[1]] if best[1] is not None else "current"
        print(f"{B}x{H}x{W}x{Ci}->{Co} k{k} s{s}: M={M} N={N} K={K}  current {cur:7.1f} us "
              f"({fl / cur / 1e6:5.0f} TF/s)  best {best[0]:7.1f} us ({fl / best[0] / 1e6:5.0f} TF/s) "
              f"tile {bt} splits {best[2]}  formula splits for that tile "
              f"{cg._tn_splits(M, N, K, best[1], dev) if best[1] is not None else '-'}", flush=True)
    print(f"sum over shapes (one call each): current {tot_cur:.0f} us  best {tot_best:.0f} us")


if __name__ == "__main__":
    main()
