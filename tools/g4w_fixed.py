"""Fixed per-tile cost of gemm4w: time vs K at M=32768, N=8192 (4096 tiles = 16 per CU), with and
without the epilogue (EPI_SKIP, measurement only), against the library at the same shapes."""
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


def run(a, b, ako, bko, trans, skip, persist=False, extra=0):
    L = G._L()
    M, Ka = (a.shape[1], a.shape[0]) if ako else (a.shape[0], a.shape[1])
    N = b.shape[1] if bko else b.shape[0]
    OM, ON = (N, M) if trans else (M, N)
    c = torch.empty(OM, ON, dtype=a.dtype, device=a.device)
    epi = (G.EPI_TRANS if trans else 0) | (128 if skip else 0) | (G.EPI_PERSIST if persist else 0) | extra

    def f():
        rc = L.pha_gemm4w(1, G._ptr(a), G._ptr(b), G._ptr(c), M, N, Ka, a.stride(0), b.stride(0), c.stride(0),
                          int(ako), int(bko), epi, G._ptr(None), G._ptr(None), 0, G._ptr(None),
                          G.sched_variant(ako, bko), G._stream(a))
        assert rc == 0, rc
    return f


r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
M, N = 32768, 8192
SHAPES = [(M, N, K) for K in (64, 256, 2048)]
if len(sys.argv) > 1:   # M,N,K triples
    SHAPES = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
for M, N, K in SHAPES:
    x, bt, w, xt = r(M, K), r(N, K), r(K, N), r(K, M)
    fl = 2.0 * M * N * K
    t = {}
    t["NT"] = timeit(run(x, bt, False, False, False, False))
    t["NT-noepi"] = timeit(run(x, bt, False, False, False, True))
    t["NNt"] = timeit(run(w, x, True, False, True, False))
    t["NNt-noepi"] = timeit(run(w, x, True, False, True, True))
    t["NT-nostore"] = timeit(run(x, bt, False, False, False, False, extra=512))
    t["NT-nostage"] = timeit(run(x, bt, False, False, False, False, extra=1024))
    t["NT-neither"] = timeit(run(x, bt, False, False, False, False, extra=1536))
    t["NT-ntstore"] = timeit(run(x, bt, False, False, False, False, extra=2048))
    t["NNt-ntstore"] = timeit(run(w, x, True, False, True, False, extra=2048))
    t["TN"] = timeit(run(xt, w, True, True, False, False))
    t["lib NT"] = timeit(lambda: x @ bt.t())
    print(f"M={M} N={N} K={K:5d}: " + "  ".join(f"{k} {v * 1e6:7.1f}us ({fl / v / 1e12:5.0f}TF)" for k, v in t.items()), flush=True)
