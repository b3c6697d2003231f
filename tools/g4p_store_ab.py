"""Where gemm4p's store cost comes from: per-CU store throughput vs a chip-wide burst (all CUs
reach their tile boundary together). Variants at one shape, interleaved rounds, median of 5:
grid 256 / 128, start stagger (groups of workgroups delayed), non-temporal stores.

  python tools/g4p_store_ab.py [M,N,K ...]
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


shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(32768, 6144, 2048)]
for M, N, K in shapes:
    x, wt = r(M, K), r(N, K)
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    var = {"lib": lambda: x @ wt.t()}
    for grid in (256, 128):
        var[f"g{grid}"] = (lambda g: lambda: G.gemm_p(x, wt, out=c, grid=g))(grid)
        var[f"g{grid}-nostore"] = (lambda g: lambda: G.gemm_p(x, wt, out=c, grid=g, epi_extra=512))(grid)
    var["nt"] = lambda: G.gemm_p(x, wt, out=c, epi_extra=2048)
    for st in (1, 4, 16):
        var[f"stagger{st}"] = (lambda v: lambda: G.gemm_p(x, wt, out=c, epi_extra=4096 | (v << 16)))(st)
        var[f"stagger{st}-nostore"] = (lambda v: lambda: G.gemm_p(x, wt, out=c, epi_extra=4096 | 512 | (v << 16)))(st)
    times = {k: [] for k in var}
    for f in var.values():
        f()
    for _ in range(5):
        for k, f in var.items():
            times[k].append(t1(f))
    fl = 2.0 * M * N * K
    print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {statistics.median(v) * 1e6:.0f}us/{fl / statistics.median(v) / 1e12:.0f}TF"
                                             for k, v in times.items()), flush=True)
