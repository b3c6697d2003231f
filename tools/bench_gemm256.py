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


def gemm8p(M, N, K, ako, bko):
    a = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16() if ako else (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16() if bko else (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    A = a.t() if ako else a
    Bm = b if bko else b.t()
    c = conv_gemm.gemm8p(a, b, ako, bko)
    ref = A.float() @ Bm.float()
    err = (c.float() - ref).abs().max().item() / ref.abs().max().item()
    fl = 2.0 * M * N * K
    t = timeit(lambda: conv_gemm.gemm8p(a, b, ako, bko))
    tl = timeit(lambda: A @ Bm)
    lay = ("T" if ako else "N") + ("N" if bko else "T")   # BLAS-style: op(A) op(B) with B^T stored = "T"
    print(f"gemm8p {lay} M={M} N={N} K={K}: {fl / t / 1e12:7.1f} TF  lib {fl / tl / 1e12:7.1f} TF  rel_err {err:.2e}",
          flush=True)


def gemm_tn(M, N, K):
    a = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    c = conv_gemm.gemm256_tn(a, b)
    ref = a.float().t() @ b.float()
    err = (c.float() - ref).abs().max().item() / ref.abs().max().item()
    fl = 2.0 * M * N * K
    t = timeit(lambda: conv_gemm.gemm256_tn(a, b))
    tl = timeit(lambda: a.t() @ b)
    print(f"gemm256_tn M={M} N={N} K={K}: {fl / t / 1e12:7.1f} TF  lib {fl / tl / 1e12:7.1f} TF  rel_err {err:.2e}",
          flush=True)


def conv_bwd(N, H, W, C, Co, k, s, p):
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(Co, C, k, k, device="cuda") * 0.05).bfloat16()
    OH = (H + 2 * p - k) // s + 1
    OW = (W + 2 * p - k) // s + 1
    dy = torch.randn(N, OH, OW, Co, device="cuda").bfloat16()
    xc = x.permute(0, 3, 1, 2).float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    TF.conv2d(xc, wf, None, s, p).backward(dy.permute(0, 3, 1, 2).float())
    dx_ref, dw_ref = xc.grad.permute(0, 2, 3, 1), wf.grad
    dx = conv_gemm.conv256_dgrad(dy, w, x.shape, (s, s), (p, p), (1, 1))
    dw = conv_gemm.conv256_wgrad(dy, x, w.shape, (s, s), (p, p), (1, 1))
    ex = (dx.float() - dx_ref).abs().max().item() / dx_ref.abs().max().item()
    ew = (dw.float() - dw_ref).abs().max().item() / dw_ref.abs().max().item()
    fl = 2.0 * N * OH * OW * Co * C * k * k
    td = timeit(lambda: conv_gemm.conv256_dgrad(dy, w, x.shape, (s, s), (p, p), (1, 1)))
    tw = timeit(lambda: conv_gemm.conv256_wgrad(dy, x, w.shape, (s, s), (p, p), (1, 1)))
    xcl = x.permute(0, 3, 1, 2)
    dycl = dy.permute(0, 3, 1, 2)
    wcl = w.contiguous(memory_format=torch.channels_last)
    cb = torch.ops.aten.convolution_backward
    tdl = timeit(lambda: cb(dycl, xcl, wcl, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False]))
    twl = timeit(lambda: cb(dycl, xcl, wcl, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False]))
    print(f"conv256 bwd N={N} {H}x{W} {C}->{Co} k{k} s{s}: dgrad {td * 1e3:.3f} ms (MIOpen {tdl * 1e3:.3f}) "
          f"wgrad {tw * 1e3:.3f} ms (MIOpen {twl * 1e3:.3f})  {fl / td / 1e12:.0f}/{fl / tw / 1e12:.0f} TF  "
          f"rel_err dx {ex:.2e} dw {ew:.2e}", flush=True)


if __name__ == "__main__":
    if "8pvar" in sys.argv[1:]:
        gemm8p(264, 520, 200, False, True)
        for shp in [(8192, 8192, 8192), (16384, 6144, 2048)]:
            for lay in [(False, False), (False, True)]:
                gemm8p(*shp, *lay)
        sys.exit(0)
    if "8p" in sys.argv[1:]:
        for lay in [(False, False), (False, True), (True, False), (True, True)]:
            gemm8p(264, 520, 200, *lay)    # ragged tiles / K tail first (correctness)
        for shp in [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 6144, 2048), (16384, 2048, 2048),
                    (16384, 8192, 2048), (16384, 2048, 8192)]:
            for lay in [(False, False), (False, True), (True, False)]:
                gemm8p(*shp, *lay)
        sys.exit(0)
    if "bwd" in sys.argv[1:]:
        for shp in [(512, 384, 1000), (2048, 2048, 16384), (2048, 8192, 16384), (8192, 2048, 16384)]:
            gemm_tn(*shp)
        for c in [(8, 9, 11, 16, 24, 3, 2, 1), (4, 10, 10, 8, 64, 7, 2, 3), (256, 56, 56, 64, 64, 1, 1, 0),
                  (256, 56, 56, 64, 64, 3, 1, 1), (256, 56, 56, 64, 256, 1, 1, 0), (256, 56, 56, 256, 64, 1, 1, 0),
                  (256, 28, 28, 128, 128, 3, 1, 1), (256, 14, 14, 256, 256, 3, 1, 1), (256, 7, 7, 512, 512, 3, 1, 1),
                  (256, 56, 56, 128, 128, 3, 2, 1), (256, 56, 56, 256, 512, 1, 2, 0),
                  (256, 14, 14, 1024, 256, 1, 1, 0), (256, 224, 224, 8, 64, 7, 2, 3)]:
            conv_bwd(*c)
        sys.exit(0)
    gemm(512, 384, 200 - 200 % 8)          # ragged tails first (correctness)
    for shp in [(4096, 4096, 4096), (16384, 2048, 2048), (16384, 8192, 2048), (16384, 2048, 8192), (8192, 8192, 8192)]:
        gemm(*shp)
    for c in [(256, 56, 56, 64, 64, 1, 1, 0), (256, 56, 56, 64, 64, 3, 1, 1), (256, 56, 56, 64, 256, 1, 1, 0),
              (256, 28, 28, 128, 128, 3, 1, 1), (256, 14, 14, 256, 256, 3, 1, 1), (256, 7, 7, 512, 512, 3, 1, 1),
              (256, 56, 56, 128, 128, 3, 2, 1), (256, 14, 14, 1024, 256, 1, 1, 0), (8, 9, 11, 16, 24, 3, 2, 1)]:
        conv(*c)
