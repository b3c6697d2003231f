"""gemm4w (one wave per SIMD, 256x256x64) vs hipBLASLt vs gemm8p: numerics against fp32 and speed
at every GEMM of a GPT-3 1.3B step (micro-batch 16: M = 32768 tokens), all in one process on
random operands."""
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402
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


def check():
    torch.manual_seed(0)
    for (M, N, K) in [(256, 256, 64), (512, 768, 192), (264, 520, 128), (1024, 2048, 512), (4096, 4096, 4096)]:
        for ako in (False, True):
            for bko in (False, True):
                a = r(K, M) if ako else r(M, K)
                b = r(K, N) if bko else r(N, K)
                A = a.float().t() if ako else a.float()
                B = b.float() if bko else b.float().t()
                ref = A @ B
                c = G.gemm(a, b, ako, bko)
                err = (c.float() - ref).abs().max().item() / ref.abs().max().item()
                print(f"check M={M} N={N} K={K} ako={int(ako)} bko={int(bko)} rel_err={err:.2e}", flush=True)
                assert err < 1e-2, err
    # epilogues
    M, N, K = 512, 768, 256
    a, b = r(M, K), r(K, N)
    bias = torch.randn(N, device="cuda")
    ref = a.float() @ b.float() + bias
    c, pre = G.gemm(a, b, False, True, bias=bias, act="gelu", aux_out=True)
    g = torch.nn.functional.gelu(ref, approximate="tanh")
    print("epi gelu err", (c.float() - g).abs().max().item(), "pre err", (pre.float() - ref).abs().max().item())
    # dgelu + colsum: dH = (dY @ W^T) * gelu'(pre)
    dY = r(M, K)
    W = r(N, K)   # B^T layout [N][K]
    dA = dY.float() @ W.float().t()
    x = pre.float().requires_grad_()
    gref = torch.autograd.grad(torch.nn.functional.gelu(x, approximate="tanh"), x, dA)[0]
    dH, part = G.gemm(dY, W, False, False, act="dgelu", aux=pre, colsum=True)
    db = G.colsum_finish(part, torch.float32)
    print("epi dgelu err", (dH.float() - gref).abs().max().item() / gref.abs().max().item(),
          "colsum err", (db - dH.float().sum(0)).abs().max().item() / dH.float().sum(0).abs().max().item(), flush=True)


def bench():
    T = 32768
    tot = {"lib": 0.0, "g4w": 0.0, "g8p": 0.0}
    for name, K, N in [("qkv", 2048, 6144), ("out", 2048, 2048), ("fc1", 2048, 8192), ("fc2", 8192, 2048)]:
        x, w, dy = r(T, K), r(K, N), r(T, N)
        fl = 2.0 * T * K * N
        for lab, f_lib, f_own, f_8p in [
            ("fwd x@W    ", lambda: x @ w, lambda: G.gemm(x, w, False, True), lambda: conv_gemm.gemm8p(x, w, False, True)),
            ("dX  dY@W^T ", lambda: dy @ w.t(), lambda: G.gemm(dy, w, False, False), lambda: conv_gemm.gemm8p(dy, w, False, False)),
            ("dW  x^T@dY ", lambda: x.t() @ dy, lambda: G.gemm(x, dy, True, True), lambda: conv_gemm.gemm8p(x, dy, True, True)),
        ]:
            tl, to, t8 = timeit(f_lib), timeit(f_own), timeit(f_8p)
            tot["lib"] += tl * 24
            tot["g4w"] += to * 24
            tot["g8p"] += t8 * 24
            print(f"{name} {lab} {T}x{N}x{K}: lib {fl / tl / 1e12:7.1f} TF  g4w {fl / to / 1e12:7.1f} TF  "
                  f"g8p {fl / t8 / 1e12:7.1f} TF   g4w/lib {tl / to:5.3f}", flush=True)
    E = r(50304, 2048)
    h, dl = r(T, 2048), r(T, 50304)
    fl = 2.0 * T * 2048 * 50304
    for lab, f_lib, f_own in [("logits h@E^T", lambda: h @ E.t(), lambda: G.gemm(h, E, False, False)),
                              ("dh dL@E     ", lambda: dl @ E, lambda: G.gemm(dl, E, False, True)),
                              ("dE dL^T@h   ", lambda: dl.t() @ h, lambda: G.gemm(dl, h, True, True))]:
        tl, to = timeit(f_lib, 5), timeit(f_own, 5)
        tot["lib"] += tl
        tot["g4w"] += to
        print(f"head {lab}: lib {fl / tl / 1e12:7.1f} TF  g4w {fl / to / 1e12:7.1f} TF   g4w/lib {tl / to:5.3f}",
              flush=True)
    # stride experiment: NT with power-of-two vs padded row strides (L2 channel / TLB effects)
    for K, pad in ((2048, 0), (2048, 64), (2048, 128), (8192, 0), (8192, 64)):
        M, N = 32768, 8192
        ab = r(M, K + pad)
        bb = r(N, K + pad)
        a, bt = ab[:, :K], bb[:, :K]
        fl = 2.0 * M * N * K
        to = timeit(lambda: G.gemm(a, bt, False, False))
        tl = timeit(lambda: a @ bt.t())
        print(f"NT stride K={K} ld={K + pad}: g4w {fl / to / 1e12:7.1f} TF  lib {fl / tl / 1e12:7.1f} TF", flush=True)
    for M in (4096, 8192):
        a, bt = r(M, M), r(M, M)
        fl = 2.0 * M ** 3
        tl, to = timeit(lambda: a @ bt.t()), timeit(lambda: G.gemm(a, bt, False, False))
        print(f"square NT {M}^3: lib {fl / tl / 1e12:7.1f} TF  g4w {fl / to / 1e12:7.1f} TF", flush=True)
    print("per-step GEMM ms (mb16): " + "  ".join(f"{k} {v * 1e3:.1f}" for k, v in tot.items()))


if __name__ == "__main__":
    check()
    if "check" not in sys.argv:
        bench()
