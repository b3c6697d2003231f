"""Own GEMM on the transposed-store layout (gemm4w A K-outer / B K-contiguous, C^T stored) vs the
library, at every GEMM of a GPT-3 1.3B step (micro-batch 16: M = 32768 tokens).

  fwd  y = x @ W          lib NN, lib NT on a cached W^T, own nn(x, W)
  dX   dX = dY @ W^T      lib NT, own NT (both K-contiguous), own nn(dY, W^T) on the cached W^T
  dW   dW = x^T @ dY      lib TN, own TN
plus a numerics check of the transposed store with every epilogue, and a SCHED sweep."""
import os
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


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


def check():
    torch.manual_seed(0)
    for (M, N, K) in [(256, 256, 64), (264, 520, 128), (1024, 2048, 512), (4096, 1536, 2048)]:
        x, w = r(M, K), r(K, N)
        ref = x.float() @ w.float()
        for P in (False,):
            c = G.nn(x, w)
            err = (c.float() - ref).abs().max().item() / ref.abs().max().item()
            print(f"check nn M={M} N={N} K={K} persistent={P} rel_err={err:.2e}", flush=True)
            assert c.shape == (M, N) and err < 1e-2, err
            bt = w.t().contiguous()
            c = G.gemm(x, bt, False, False)
            err = (c.float() - ref).abs().max().item() / ref.abs().max().item()
            print(f"check NT M={M} N={N} K={K} persistent={P} rel_err={err:.2e}", flush=True)
            assert err < 1e-2, err
    M, N, K = 520, 768, 256
    x, w = r(M, K), r(K, N)
    bias = torch.randn(N, device="cuda")
    ref = x.float() @ w.float() + bias
    c, pre = G.nn(x, w, bias=bias, act="gelu", aux_out=True)
    g = torch.nn.functional.gelu(ref, approximate="tanh")
    e1 = (c.float() - g).abs().max().item()
    e2 = (pre.float() - ref).abs().max().item()
    print(f"check nn bias+gelu err {e1:.3e} pre err {e2:.3e}", flush=True)
    assert e1 < 0.1 and e2 < 0.1
    # dgelu + colsum on the transposed store: dH = (dY @ W^T) * gelu'(pre), db = colsum(dH)
    dy = r(M, N)
    wt = w.t().contiguous()          # dY [M, N] @ W^T [N, K]
    pre2 = r(M, K)
    dh, part = G.nn(dy, wt, act="dgelu", aux=pre2, colsum=True)
    xg = pre2.float().requires_grad_()
    gref = torch.autograd.grad(torch.nn.functional.gelu(xg, approximate="tanh"), xg, dy.float() @ w.float().t())[0]
    e3 = (dh.float() - gref).abs().max().item() / gref.abs().max().item()
    db = G.colsum_finish(part, torch.float32)
    e4 = (db - dh.float().sum(0)).abs().max().item() / dh.float().sum(0).abs().max().item()
    print(f"check nn dgelu err {e3:.3e} colsum err {e4:.3e}", flush=True)
    assert e3 < 2e-2 and e4 < 1e-2


def bench():
    T = 32768
    tot = {"lib": 0.0, "own": 0.0}
    for name, K, N in [("qkv", 2048, 6144), ("out", 2048, 2048), ("fc1", 2048, 8192), ("fc2", 8192, 2048)]:
        x, w, dy = r(T, K), r(K, N), r(T, N)
        wt = w.t().contiguous()
        b_ = torch.randn(N, device="cuda")
        fl = 2.0 * T * K * N
        rows = [
            ("fwd", [("lib NN", lambda: x @ w), ("lib NT(Wt)", lambda: x @ wt.t())],
             [("own nn", lambda: G.nn(x, w)),
              ("own nn+bias+gelu", lambda: G.nn(x, w, bias=b_, act="gelu", aux_out=True))]),
            ("dX ", [("lib NT", lambda: dy @ w.t())],
             [("own NT", lambda: G.gemm(dy, w, False, False)),
              ("own nn(Wt)", lambda: G.nn(dy, wt))]),
            ("dW ", [("lib TN", lambda: x.t() @ dy)], [("own TN", lambda: G.gemm(x, dy, True, True))]),
        ]
        for lab, libs, owns in rows:
            res = [(n, timeit(f)) for n, f in libs + owns]
            bl = min(t for n, t in res[:len(libs)])
            bo = min(t for n, t in res[len(libs):])
            tot["lib"] += bl * 24
            tot["own"] += bo * 24
            print(f"{name} {lab} {T}x{N}x{K}: " + "  ".join(f"{n} {fl / t / 1e12:6.0f}" for n, t in res) +
                  f"  TF   best own/lib {bl / bo:5.3f}", flush=True)
    E = r(50304, 2048)
    h, dl = r(T, 2048), r(T, 50304)
    fl = 2.0 * T * 2048 * 50304
    for lab, f_lib, f_own in [("logits h@E^T", lambda: h @ E.t(), lambda: G.gemm(h, E, False, False)),
                              ("dh dL@E     ", lambda: dl @ E, lambda: G.nn(dl, E)),
                              ("dE dL^T@h   ", lambda: dl.t() @ h, lambda: G.gemm(dl, h, True, True))]:
        tl, to = timeit(f_lib, 5), timeit(f_own, 5)
        if not lab.startswith("logits np"):
            tot["lib"] += tl
            tot["own"] += to
        print(f"head {lab}: lib {fl / tl / 1e12:6.0f} TF  own {fl / to / 1e12:6.0f} TF   own/lib {tl / to:5.3f}",
              flush=True)
    print("per-step GEMM ms (mb16, best of each side): " + "  ".join(f"{k} {v * 1e3:.1f}" for k, v in tot.items()))


def sweep():
    """SCHED variants of the NT and transposed-store layouts at the GPT shapes"""
    T = 32768
    for K, N in ((2048, 8192), (2048, 2048), (8192, 2048)):
        x, w, bt = r(T, K), r(K, N), r(N, K)
        fl = 2.0 * T * K * N
        out = []
        for sc in ("0", "2"):
            os.environ["PHA_G4W_SCHED"] = sc
            out.append(f"nn sched{sc} {fl / timeit(lambda: G.nn(x, w)) / 1e12:6.0f}")
            out.append(f"NT sched{sc} {fl / timeit(lambda: G.gemm(x, bt, False, False)) / 1e12:6.0f}")
        os.environ.pop("PHA_G4W_SCHED", None)
        print(f"nn sweep {T}x{N}x{K}: " + "  ".join(out) + " TF", flush=True)


if __name__ == "__main__":
    check()
    if "check" not in sys.argv:
        bench()
        sweep()
