"""Every GEMM of a GPT-3 1.3B training step (M = 8 x 2048 tokens) in its real operand layout:
hipBLASLt through torch (as the model calls it) vs the own 8-phase kernel (gemm8p)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import conv_gemm  # noqa: E402


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


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


T = 16384
total_lib = total_own = 0.0
for name, K, N in [("qkv", 2048, 6144), ("out", 2048, 2048), ("fc1", 2048, 8192), ("fc2", 8192, 2048)]:
    x, w, dy = r(T, K), r(K, N), r(T, N)
    fl = 2.0 * T * K * N
    cases = [
        ("fwd  x@W    ", lambda: x @ w, lambda: conv_gemm.gemm8p(x, w, False, True)),
        ("dX   dY@W^T ", lambda: dy @ w.t(), lambda: conv_gemm.gemm8p(dy, w, False, False)),
        ("dW   x^T@dY ", lambda: x.t() @ dy, lambda: conv_gemm.gemm8p(x, dy, True, True)),
    ]
    tp = timeit(lambda: conv_gemm.weight_grad(x, dy))
    print(f"{name} dW picked (lib / own / own split-K): {fl / tp / 1e12:7.1f} TF ({tp * 1e3:.3f} ms) "
          f"choice={conv_gemm._gemm_pick.get(('dw', x.dtype, T, K, N))}", flush=True)
    for lab, f_lib, f_own in cases:
        tl, to = timeit(f_lib), timeit(f_own)
        total_lib += tl * 24
        total_own += min(tl, to) * 24
        print(f"{name} {lab} {T}x{N}x{K}: lib {fl / tl / 1e12:7.1f} TF ({tl * 1e3:.3f} ms)  own {fl / to / 1e12:7.1f} TF "
              f"({to * 1e3:.3f} ms)", flush=True)
E = r(50304, 2048)
h, dl = r(T, 2048), r(T, 50304)
fl = 2.0 * T * 2048 * 50304
for lab, f_lib, f_own in [("logits h@E^T", lambda: h @ E.t(), lambda: conv_gemm.gemm8p(h, E, False, False)),
                          ("dh dL@E     ", lambda: dl @ E, lambda: conv_gemm.gemm8p(dl, E, False, True)),
                          ("dE dL^T@h   ", lambda: dl.t() @ h, lambda: conv_gemm.gemm8p(dl, h, True, True))]:
    tl, to = timeit(f_lib), timeit(f_own)
    total_lib += tl
    total_own += min(tl, to)
    print(f"head {lab} : lib {fl / tl / 1e12:7.1f} TF ({tl * 1e3:.3f} ms)  own {fl / to / 1e12:7.1f} TF ({to * 1e3:.3f} ms)",
          flush=True)
print(f"per-step GEMM time: all hipBLASLt {total_lib * 1e3:.1f} ms, best-of-both {total_own * 1e3:.1f} ms")
