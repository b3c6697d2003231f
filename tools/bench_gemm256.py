"""Numerics + speed of the 256-row-tile glds GEMM / conv (gemm256.hip) vs hipBLASLt / MIOpen,
on random bf16 operands in one process."""
import sys
import time

import torch
import torch.nn.functional as TF

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import conv_gemm  # noqa: E402


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


def gemm(M, N, K):
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    bt = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    c = conv_gemm.gemm256_nt(a, bt)
    ref = a.float() @ bt.float().t()
    err = (c.float() - ref).abs().max().item() / ref.abs().max().item()
    fl = 2.0 * M * N * K
    t = timeit(lambda: conv_gemm.gemm256_nt(a, bt))
    tl = timeit(lambda: a @ bt.t())
    print(f"gemm256 M={M} N={N} K={K}: {fl / t / 1e12:7.1f} TF  lib {fl / tl / 1e12:7.1f} TF  rel_err {err:.2e}",
          flush=True)


def conv(N, H, W, C, Co, k, s, p):
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(Co, C, k, k, device="cuda") * 0.05).bfloat16()
    wk = w.permute(0, 2, 3, 1).contiguous()
    y = conv_gemm.conv256_fwd(x, wk, (s, s), (p, p), (1, 1))
    xc = x.permute(0, 3, 1, 2)
    ref = TF.conv2d(xc.float(), w.float(), None, s, p).permute(0, 2, 3, 1)
    err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
    OH = (H + 2 * p - k) // s + 1
    fl = 2.0 * N * OH * OH * Co * C * k * k
    t = timeit(lambda: conv_gemm.conv256_fwd(x, wk, (s, s), (p, p), (1, 1)))
    xcl = xc.contiguous(memory_format=torch.channels_last)
    tl = timeit(lambda: TF.conv2d(xcl, w, None, s, p))
    print(f"conv256 N={N} {H}x{W} {C}->{Co} k{k} s{s}: fwd {fl / t / 1e12:6.1f} TF ({t * 1e3:.3f} ms)  "
          f"MIOpen {fl / tl / 1e12:6.1f} TF ({tl * 1e3:.3f} ms)  rel_err {err:.2e}", flush=True)


if __name__ == "__main__":
    gemm(512, 384, 200 - 200 % 8)          # ragged tails first (correctness)
    for shp in [(4096, 4096, 4096), (16384, 2048, 2048), (16384, 8192, 2048), (16384, 2048, 8192), (8192, 8192, 8192)]:
        gemm(*shp)
    for c in [(256, 56, 56, 64, 64, 1, 1, 0), (256, 56, 56, 64, 64, 3, 1, 1), (256, 56, 56, 64, 256, 1, 1, 0),
              (256, 28, 28, 128, 128, 3, 1, 1), (256, 14, 14, 256, 256, 3, 1, 1), (256, 7, 7, 512, 512, 3, 1, 1),
              (256, 56, 56, 128, 128, 3, 2, 1), (256, 14, 14, 1024, 256, 1, 1, 0), (8, 9, 11, 16, 24, 3, 2, 1)]:
        conv(*c)
