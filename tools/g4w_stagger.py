"""Store-burst study of gemm4w: every CU ends its tile at the same moment and writes 128 KB, so
at M=32768, N=8192 the whole 512 MB output goes out in 16 chip-wide bursts that are not overlapped
with any compute (tools/g4w_fixed.py: NT 902 us vs 708 us without stores). EPI_STAGGER delays the
first-round workgroups in phase groups so the bursts of different CUs fall at different times.
Sweeps (groups, sleep units) at K=2048 for NT and the transposed-store NN, against the library."""
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402

EPI_STAGGER = 4096


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
shapes = [(32768, 8192, 2048), (32768, 2048, 8192), (32768, 6144, 2048), (32768, 2048, 2048)]
for M, N, K in shapes:
    x, bt, w = r(M, K), r(N, K), r(K, N)
    fl = 2.0 * M * N * K
    ref = x @ bt.t()
    t = {"lib": timeit(lambda: x @ bt.t())}
    for groups, units in ((1, 0), (2, 3), (2, 6), (4, 1), (4, 2), (4, 3), (4, 4), (8, 1), (8, 2)):
        extra = 0 if units == 0 else (EPI_STAGGER | (units << 16) | (groups << 24))
        f, c = run(x, bt, False, False, False, extra)
        t[f"NT g{groups}u{units}"] = timeit(f)
        if units == 0 or (groups, units) == (4, 2):
            f()
            torch.cuda.synchronize()
            err = (c.float() - ref.float()).abs().max().item()
            assert err < 0.5, err
        f, c = run(w, x, True, False, True, extra)
        t[f"NNt g{groups}u{units}"] = timeit(f)
    print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {v * 1e6:6.1f}us ({fl / v / 1e12:5.0f})" for k, v in t.items()),
          flush=True)
