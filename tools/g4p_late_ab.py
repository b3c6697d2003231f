"""gemm4p late-wait variants (EPI_LATE_SHIFT bits, csrc/kernels/gemm4p.hip lv_lwg / lv_ldma) on the
GPT-3 1.3B NT products: bitwise comparison with the EARLY schedule, then interleaved timing (median
of 5) of every variant and hipBLASLt.  python tools/g4p_late_ab.py"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402

T = 32768
LVS = [int(v) for v in os.environ.get("LVS", "0,8,10,11,13").split(",")]


def t1(fn, iters=8):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


def main():
    tot = {}
    for name, N, K in (("fc2 fwd", 2048, 8192), ("qkv dX", 2048, 6144), ("qkv fwd", 6144, 2048),
                       ("out fwd", 2048, 2048), ("fc2 dX", 8192, 2048), ("head", 50304, 2048)):
        x, wt, b = r(T, K), r(N, K), torch.randn(N, device="cuda")
        fl = 2.0 * T * N * K
        var = {f"lv{lv}": (lambda lv=lv: G.gemm_p(x, wt, bias=b, epi_extra=G.EPI_EARLY | (lv << 17))) for lv in LVS}
        var["lib"] = lambda: torch.addmm(b.bfloat16(), x, wt.t())
        ref = var["lv0"]().clone()
        eq = {k: torch.equal(ref, f()) for k, f in var.items() if k != "lib"}
        times = {k: [] for k in var}
        for _ in range(5):
            for k, fn in var.items():
                times[k].append(t1(fn))
        med = {k: statistics.median(v) for k, v in times.items()}
        for k, v in med.items():
            tot[k] = tot.get(k, 0.0) + v
        print(f"NT {name} {T}x{N}x{K}: " + "  ".join(f"{k} {med[k] * 1e6:.0f}us/{fl / med[k] / 1e12:.0f}TF" for k in var)
              + f"  bitwise={all(eq.values())} {'' if all(eq.values()) else eq}", flush=True)
    print("sum: " + "  ".join(f"{k} {v * 1e3:.2f}ms" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
