"""DMA placement in the NT gemm4p K-loop (SPREAD, gemm4p.hip sp_na / sp_gb): the 16 LDS-DMAs of
the next-next K-tile over 16 consecutive MFMA groups (LV 8, shipped) vs spread over 24-28 groups
(LV 40 / 72 / 104), plus the s_memtime-stamped builds (LV 15 / 47), on the GPT-3 1.3B NT shapes at
micro-batch 48 (M = 98,304) after a sustained warm-up; hipBLASLt (-1) on the same operands.
python tools/g4p_spread.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402

T = int(os.environ.get("STAMP_M", 98304))


def epi_of(lv):
    return G.EPI_EARLY | G.EPI_BIAS | ((lv & 15) << 17) | (((lv >> 5) & 3) << 28)


def main():
    L = G._L()
    plain = [int(v) for v in os.environ.get("LVS", "8,40,72,104,-1").split(",")]
    stamped = [int(v) for v in os.environ.get("STAMPED", "15,47").split(",") if v]
    for name, N, K in (("fc2 fwd", 2048, 8192), ("qkv dX", 2048, 6144), ("qkv fwd", 6144, 2048),
                       ("out fwd", 2048, 2048), ("fc2 dX", 8192, 2048)):
        x = torch.randn(T, K, device="cuda").bfloat16()
        wt = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        b = torch.randn(N, device="cuda") * 0.02
        c = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        grid = G._num_cus(x.device)
        ws = torch.zeros(grid * 4 * 4, dtype=torch.int64, device="cuda")
        bb = b.bfloat16()

        def run(lv, w=None):
            if lv < 0:
                torch.addmm(bb, x, wt.t(), out=c)
                return
            rc = L.pha_gemm4p(G._DT[x.dtype], G._ptr(x), G._ptr(wt), G._ptr(c), T, N, K, K, K, N, 0, 0, 0,
                              epi_of(lv), G._ptr(b), grid, G._group_m(False, False, K, N), G._ptr(w),
                              1, G._stream(x), None)
            assert rc == 0, rc
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 1.0:
            for _ in range(8):
                run(8)
            torch.cuda.synchronize()
        res = {}
        for _ in range(3):
            for lv in plain + stamped:
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(10):
                    run(lv, ws if lv in stamped else None)
                torch.cuda.synchronize()
                res.setdefault(lv, []).append((time.perf_counter() - t1) / 10)
        ref = torch.addmm(bb, x, wt.t()).float()
        fl = 2.0 * T * N * K
        line = f"NT {name} {T}x{N}x{K}: " + "  ".join(
            f"lv{lv} {min(res[lv]) * 1e6:.0f}us/{fl / min(res[lv]) / 1e12:.0f}TF" for lv in plain + stamped)
        errs = []
        for lv in plain:
            c.zero_()
            run(lv)
            torch.cuda.synchronize()
            errs.append(f"lv{lv} {(c.float() - ref).abs().max().item():.3g}")
        print(line + "  max|err| " + " ".join(errs), flush=True)
        for lv in stamped:
            ws.zero_()
            run(lv, ws)
            torch.cuda.synchronize()
            a = ws.view(grid, 4, 4).cpu().numpy().astype(np.float64)
            tot, ab, rel, n = a[..., 0], a[..., 1], a[..., 2], np.maximum(a[..., 3], 1)
            print(f"   lv{lv} per K-tile (median over waves, shader cycles): total {np.median(tot / n):.0f}  "
                  f"A/B wait {np.median(ab / n):.0f}  release wait {np.median(rel / n):.0f}  "
                  f"rest {np.median((tot - ab - rel) / n):.0f} (ideal 2048)", flush=True)
        del x, wt, c


if __name__ == "__main__":
    main()
