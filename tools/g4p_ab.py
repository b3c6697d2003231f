"""gemm4p A/B at one GEMM shape: the persistent main loop without any epilogue (EPI_SKIP), with the
epilogue but stores dropped (EPI_NOSTORE), the full kernel, per GROUP_M, against gemm4w with and
without its epilogue and the library. Interleaved rounds in one process, median of 5.

  python tools/g4p_ab.py [M,N,K ...]
"""
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402


def t1(fn, iters=10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(32768, 6144, 2048), (32768, 2048, 8192)]
for M, N, K in shapes:
    x, wt = r(M, K), r(N, K)
    L = G._L()
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")

    def g4w(epi):
        return lambda: L.pha_gemm4w(1, G._ptr(x), G._ptr(wt), G._ptr(c), M, N, K, K, K, N, 0, 0, epi, G._ptr(None),
                                    G._ptr(None), 0, G._ptr(None), 2, G._stream(x))
    var = {
        "lib": lambda: x @ wt.t(),
        "g4w": g4w(0),
        "g4w-noepi": g4w(128),
        "g4p": lambda: G.gemm_p(x, wt, out=c),
        "g4p-nostore": lambda: G.gemm_p(x, wt, out=c, epi_extra=512),
        "g4p-noepi": lambda: G.gemm_p(x, wt, out=c, epi_extra=128),
        "g4p-rounds": lambda: G.gemm_p(x, wt, out=c, epi_extra=8192),
        "g4p-rounds-noepi": lambda: G.gemm_p(x, wt, out=c, epi_extra=8192 | 128),
        "g4p-temporal": lambda: G.gemm_p(x, wt, out=c, epi_extra=16384),
        "g4p-1tile/wg-noepi": lambda: G.gemm_p(x, wt, out=c, epi_extra=128, grid=(M // 256) * (N // 256)),
    }
    for gm in (2, 8):
        var[f"g4p-gm{gm}"] = (lambda g: lambda: G.gemm_p(x, wt, out=c, group_m=g))(gm)
    times = {k: [] for k in var}
    for f in var.values():
        f()
    for _ in range(5):
        for k, f in var.items():
            times[k].append(t1(f))
    fl = 2.0 * M * N * K
    print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {statistics.median(v) * 1e6:.0f}us/{fl / statistics.median(v) / 1e12:.0f}TF"
                                             for k, v in times.items()), flush=True)
