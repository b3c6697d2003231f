"""Micro-benchmark: our MFMA GEMM / implicit-GEMM conv vs the library path (hipBLASLt / MIOpen)
on the same random bf16 operands, interleaved rounds in one process."""
import sys
import time

import torch
import torch.nn.functional as TF

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import conv_gemm  # noqa: E402
from paddle_hackathon_amd.nn.functional.conv import _hip_conv2d  # noqa: E402


def timeit(fn, iters=20):
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


def gemm_case(M, N, K, ta=False, tb=False):
    a = (torch.rand((K, M) if ta else (M, K), device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand((N, K) if tb else (K, N), device="cuda") * 2 - 1).to(torch.bfloat16)
    fl = 2.0 * M * N * K
    t_ours = timeit(lambda: conv_gemm.matmul(a, b, ta, tb))
    t_lib = timeit(lambda: (a.t() if ta else a) @ (b.t() if tb else b))
    print(f"gemm M={M:6d} N={N:6d} K={K:6d} ta={int(ta)} tb={int(tb)}: ours {fl / t_ours / 1e12:7.1f} TF  "
          f"lib {fl / t_lib / 1e12:7.1f} TF  ratio {t_lib / t_ours:5.2f}", flush=True)


def conv_case(N, H, W, Ci, Co, k, s, p):
    x = torch.randn(N, H, W, Ci, device="cuda").to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(Co, Ci, k, k, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_(True)
    xc = x.detach().permute(0, 3, 1, 2).requires_grad_(True)  # channels_last view
    OH = (H + 2 * p - k) // s + 1
    fl = 2.0 * N * OH * OH * Co * Ci * k * k
    gy = torch.randn(N, OH, OH, Co, device="cuda").to(torch.bfloat16)

    def ours():
        y = _hip_conv2d(x, w, None, [s, s], [p, p], [1, 1], 1)
        y.backward(gy)

    def lib():
        y = TF.conv2d(xc, w, None, s, p)
        y.backward(gy.permute(0, 3, 1, 2))

    t_o, t_l = timeit(ours, 5), timeit(lib, 5)
    print(f"conv N={N} {H}x{W} {Ci}->{Co} k{k} s{s}: fwd+bwd ours {3 * fl / t_o / 1e12:6.1f} TF ({t_o * 1e3:.3f} ms)  "
          f"lib {3 * fl / t_l / 1e12:6.1f} TF ({t_l * 1e3:.3f} ms)", flush=True)


if __name__ == "__main__":
    for shp in [(4096, 4096, 4096), (16384, 2048, 2048), (16384, 8192, 2048), (16384, 2048, 8192)]:
        gemm_case(*shp)
    gemm_case(16384, 2048, 2048, tb=True)
    gemm_case(2048, 2048, 16384, ta=True)
    for c in [(256, 56, 56, 64, 64, 1, 1, 0), (256, 56, 56, 64, 64, 3, 1, 1), (256, 56, 56, 64, 256, 1, 1, 0),
              (256, 28, 28, 128, 128, 3, 1, 1), (256, 14, 14, 256, 256, 3, 1, 1), (256, 7, 7, 512, 512, 3, 1, 1),
              (256, 56, 56, 128, 128, 3, 2, 1), (256, 14, 14, 1024, 256, 1, 1, 0)]:
        conv_case(*c)
