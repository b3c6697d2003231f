"""L2-panel grouping study of gemm4w: GROUP_M (row panels walked together inside an XCD's share of
the tiles) at the GPT shapes where the own kernel trails the library, esp. the K=8192 fc2 forward
whose main loop alone runs below the K=2048 rate."""
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters)
    return best


def run(a, b, ako, bko, trans, extra=0):
    L = G._L()
    M, Ka = (a.shape[1], a.shape[0]) if ako else (a.shape[0], a.shape[1])
    N = b.shape[1] if bko else b.shape[0]
    OM, ON = (N, M) if trans else (M, N)
    c = torch.empty(OM, ON, dtype=a.dtype, device=a.device)
    epi = (G.EPI_TRANS if trans else 0) | extra

    def f():
        rc = L.pha_gemm4w(1, G._ptr(a), G._ptr(b), G._ptr(c), M, N, Ka, a.stride(0), b.stride(0), c.stride(0),
                          int(ako), int(bko), epi, G._ptr(None), G._ptr(None), 0, G._ptr(None),
                          G.sched_variant(ako, bko), G._stream(a))
        assert rc == 0, rc
    return f, c


r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
if len(sys.argv) > 1 and sys.argv[1] == "tn":   # weight-gradient layout: dW[M,N] = X^T dY, both K-outer
    for M, N, K in [(2048, 6144, 32768), (2048, 2048, 32768), (2048, 8192, 32768), (8192, 2048, 32768),
                    (2048, 50304, 32768)]:
        xt, dy = r(K, M), r(K, N)
        fl = 2.0 * M * N * K
        t = {"lib TN": timeit(lambda: xt.t() @ dy)}
        for lg in (0, 1, 2, 4, 5):
            f, c = run(xt, dy, True, True, False, lg << 28)
            t[f"TN gm{1 << lg if lg else 8}"] = timeit(f)
            if lg == 2 and N <= 8192:
                f()
                torch.cuda.synchronize()
                ref = (xt.t().float() @ dy.float())
                assert (c.float() - ref).abs().max().item() < 2.0
        print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {v * 1e6:6.1f}us ({fl / v / 1e12:5.0f})" for k, v in t.items()),
              flush=True)
    sys.exit(0)
for M, N, K in [(32768, 2048, 8192), (32768, 8192, 2048), (32768, 6144, 2048), (32768, 2048, 2048)]:
    x, bt, w = r(M, K), r(N, K), r(K, N)
    fl = 2.0 * M * N * K
    ref = x @ bt.t()
    t = {"lib NT": timeit(lambda: x @ bt.t()), "lib NN": timeit(lambda: x @ w)}
    for lg in (0, 1, 2, 4, 5, 6):
        extra = lg << 28
        f, c = run(x, bt, False, False, False, extra)
        t[f"NT gm{1 << lg if lg else 8}"] = timeit(f)
        if lg == 2:
            f()
            torch.cuda.synchronize()
            assert (c.float() - ref.float()).abs().max().item() < 0.5
        f, c = run(w, x, True, False, True, extra)
        t[f"NNt gm{1 << lg if lg else 8}"] = timeit(f)
    print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {v * 1e6:6.1f}us ({fl / v / 1e12:5.0f})" for k, v in t.items()),
          flush=True)
