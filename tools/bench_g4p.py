"""Persistent epilogue-overlapped GEMM (gemm4p) vs gemm4w vs hipBLASLt: numerics against fp32 and
speed at every GEMM of a GPT-3 1.3B step (M = 32768 tokens), one process, random operands.

  python tools/bench_g4p.py            # check + bench
  python tools/bench_g4p.py check      # numerics only
"""
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
    for (M, N, K) in [(256, 256, 64), (512, 768, 192), (264, 520, 128), (1032, 2056, 512), (4096, 4096, 1024),
                      (8, 8, 64), (2048, 6144, 256)]:
        for grid in (0, 3):
            for lay in ("nt", "tn", "nn"):
                if lay == "nt":
                    a, b = r(M, K), r(N, K)
                    ref = a.float() @ b.float().t()
                    bias = torch.randn(N, device="cuda")
                    c = G.gemm_p(a, b, False, False, grid=grid)
                    cb = G.gemm_p(a, b, False, False, bias=bias, grid=grid)
                    refb = ref + bias
                elif lay == "tn":
                    a, b = r(K, M), r(K, N)
                    ref = a.float().t() @ b.float()
                    bias = torch.randn(N, device="cuda")
                    c = G.gemm_p(a, b, True, True, grid=grid)
                    cb = G.gemm_p(a, b, True, True, bias=bias, grid=grid)
                    refb = ref + bias
                else:
                    x, w = r(M, K), r(K, N)
                    ref = x.float() @ w.float()
                    bias = torch.randn(N, device="cuda")
                    c = G.nn_p(x, w, grid=grid)
                    cb = G.nn_p(x, w, bias=bias, grid=grid)
                    refb = ref + bias
                err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
                errb = ((cb.float() - refb).abs().max() / refb.abs().max()).item()
                print(f"check {lay} M={M} N={N} K={K} grid={grid or 'cu'} rel_err={err:.2e} bias_err={errb:.2e}",
                      flush=True)
                assert err < 1e-2 and errb < 1e-2, (err, errb)
    # split-K weight gradients (fp32 slabs + in-order reduce), with bias
    for (M, N, K, sp) in [(2048, 2048, 4096, 4), (264, 520, 1024, 2), (2048, 6144, 2048, 2)]:
        a, b = r(K, M), r(K, N)
        bias = torch.randn(N, device="cuda")
        ref = a.float().t() @ b.float() + bias
        c = G.gemm_p(a, b, True, True, bias=bias, splits=sp)
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        print(f"check tn split-K M={M} N={N} K={K} splits={sp} rel_err={err:.2e}", flush=True)
        assert err < 1e-2, err
        assert torch.equal(c, G.gemm_p(a, b, True, True, bias=bias, splits=sp))
    # out-of-place strided output (ldc > N): the columns past N must stay untouched
    a, b = r(520, 256), r(264, 256)
    big = torch.full((520, 512), 7.0, device="cuda", dtype=torch.bfloat16)
    G.gemm_p(a, b, False, False, out=big[:, :264])
    assert (big[:, 264:] == 7.0).all()
    ref = a.float() @ b.float().t()
    assert ((big[:, :264].float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    print("check strided output ok", flush=True)


def bench():
    T = 32768
    tot = {"lib": 0.0, "g4w": 0.0, "g4p": 0.0}
    for name, K, N in [("qkv", 2048, 6144), ("out", 2048, 2048), ("fc1", 2048, 8192), ("fc2", 8192, 2048)]:
        x, wt, dy, w = r(T, K), r(N, K), r(T, N), r(K, N)
        fl = 2.0 * T * K * N
        rows = [
            ("fwd x@W^T   ", lambda: x @ wt.t(), lambda: G.gemm(x, wt, False, False),
             lambda: G.gemm_p(x, wt, False, False)),
            ("dX  dY@W^T  ", lambda: dy @ w.t(), lambda: G.gemm(dy, w, False, False),
             lambda: G.gemm_p(dy, w, False, False)),
            ("dW  x^T@dY  ", lambda: x.t() @ dy, lambda: G.gemm(x, dy, True, True),
             lambda: G.gemm_p(x, dy, True, True)),
        ]
        for lab, f_lib, f_4w, f_4p in rows:
            tl, t4w, t4p = timeit(f_lib), timeit(f_4w), timeit(f_4p)
            tot["lib"] += tl * 24
            tot["g4w"] += t4w * 24
            tot["g4p"] += t4p * 24
            print(f"{name} {lab} {T}x{N}x{K}: lib {fl / tl / 1e12:6.0f} TF  g4w {fl / t4w / 1e12:6.0f} TF  "
                  f"g4p {fl / t4p / 1e12:6.0f} TF", flush=True)
    # logits and their gradients (vocab 50304)
    V, H = 50304, 2048
    x, E, dl = r(T, H), r(V, H), r(T, V)
    fl = 2.0 * T * V * H
    for lab, f_lib, f_4w, f_4p in [
        ("logits x@E^T", lambda: x @ E.t(), lambda: G.gemm(x, E, False, False), lambda: G.gemm_p(x, E, False, False)),
        ("dh  dL@E    ", lambda: dl @ E, lambda: G.nn(dl, E), lambda: G.nn_p(dl, E)),
        ("dE  dL^T@x  ", lambda: dl.t() @ x, lambda: G.gemm(dl, x, True, True), lambda: G.gemm_p(dl, x, True, True)),
    ]:
        tl, t4w, t4p = timeit(f_lib, 3), timeit(f_4w, 3), timeit(f_4p, 3)
        tot["lib"] += tl
        tot["g4w"] += t4w
        tot["g4p"] += t4p
        print(f"head {lab} {T}x{V}x{H}: lib {fl / tl / 1e12:6.0f} TF  g4w {fl / t4w / 1e12:6.0f} TF  "
              f"g4p {fl / t4p / 1e12:6.0f} TF", flush=True)
    # the overlap itself: stores dropped by the bounds check (measurement only)
    x, wt = r(T, 2048), r(6144, 2048)
    t_full = timeit(lambda: G.gemm_p(x, wt, False, False))
    t_nost = timeit(lambda: G.gemm_p(x, wt, False, False, epi_extra=512))
    print(f"qkv fwd g4p with stores {t_full * 1e6:.1f} us, stores dropped {t_nost * 1e6:.1f} us", flush=True)
    print("per-step GEMM ms (same products): " + "  ".join(f"{k} {v * 1e3:.1f}" for k, v in tot.items()), flush=True)




def paths():
    """the dispatch functions the GPT step calls (ops/gemm.py mm_nt / mm_nt_bias / mm_tn), own vs
    library, per GPT-1.3B shape (B16 x S2048 tokens, 24 layers)"""
    import os
    T = 32768
    tot = {"own": 0.0, "library": 0.0}

    def both(f, iters=10):
        res = {}
        for impl in ("own", "library"):
            os.environ["PHA_GEMM_IMPL"] = impl
            res[impl] = timeit(f, iters)
        return res

    shapes = [("qkv", 2048, 6144), ("out", 2048, 2048), ("fc1", 2048, 8192), ("fc2", 8192, 2048)]
    for name, K, N in shapes:
        x, wt, w, dy = r(T, K), r(N, K), r(K, N), r(T, N)
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * K * N
        for lab, f in [("fwd mm_nt_bias", lambda: G.mm_nt_bias(x, wt, b)),
                       ("dX  mm_nt     ", lambda: G.mm_nt(dy, w)),
                       ("dW  mm_tn     ", lambda: G.mm_tn(x, dy))]:
            t = both(f)
            for k in tot:
                tot[k] += t[k] * 24
            print(f"{name} {lab} {T}x{N}x{K}: own {fl / t['own'] / 1e12:6.0f} TF  lib {fl / t['library'] / 1e12:6.0f} TF"
                  f"  ({(t['own'] / t['library'] - 1) * 100:+.1f}%)", flush=True)
    V, H = 50304, 2048
    x, E, dl = r(T, H), r(V, H), r(T, V)
    fl = 2.0 * T * V * H
    for lab, f in [("logits mm_nt", lambda: G.mm_nt(x, E)), ("dh mm_nn    ", lambda: G.mm_nn(dl, E)),
                   ("dE mm_tn    ", lambda: G.mm_tn(dl, x))]:
        t = both(f, 3)
        for k in tot:
            tot[k] += t[k]
        print(f"head {lab} {T}x{V}x{H}: own {fl / t['own'] / 1e12:6.0f} TF  lib {fl / t['library'] / 1e12:6.0f} TF"
              f"  ({(t['own'] / t['library'] - 1) * 100:+.1f}%)", flush=True)
    print("per-step GEMM ms: " + "  ".join(f"{k} {v * 1e3:.1f}" for k, v in tot.items()), flush=True)


def nnform():
    """x @ W and dY @ W^T as the NN-form kernel (K-outer weight operand, transposed store) vs the
    own NT kernel vs hipBLASLt NT, per GPT-1.3B shape"""
    T = 32768
    tot = {"lib": 0.0, "nt": 0.0, "nn": 0.0}
    for name, K, N in [("qkv", 2048, 6144), ("out", 2048, 2048), ("fc1", 2048, 8192), ("fc2", 8192, 2048),
                       ("head", 2048, 50304)]:
        x, wt, dy = r(T, K), r(N, K), r(T, N)
        w = wt.t().contiguous()
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * K * N
        ref = (x.float() @ w.float() + b.float())
        err = ((G.nn_p(x, w, bias=b).float() - ref).abs().max() / ref.abs().max()).item()
        n = 24 if name != "head" else 1
        for lab, fs in [("fwd", {"lib": lambda: torch.addmm(b, x, wt.t()), "nt": lambda: G.gemm_p(x, wt, False, False, bias=b),
                                 "nn": lambda: G.nn_p(x, w, bias=b)}),
                        ("dX ", {"lib": lambda: dy @ wt, "nt": lambda: G.gemm_p(dy, w, False, False),
                                 "nn": lambda: G.nn_p(dy, wt)})]:
            t = {k: timeit(f, 10 if n > 1 else 3) for k, f in fs.items()}
            for k in tot:
                tot[k] += t[k] * n
            print(f"{name} {lab} {T}x{N if lab == 'fwd' else K}x{K if lab == 'fwd' else N}: "
                  + "  ".join(f"{k} {fl / v / 1e12:6.0f} TF" for k, v in t.items())
                  + f"  (nn vs lib {(t['nn'] / t['lib'] - 1) * 100:+.1f}%)  fwd err {err:.1e}", flush=True)
    print("per-step ms: " + "  ".join(f"{k} {v * 1e3:.1f}" for k, v in tot.items()), flush=True)


def gelu():
    """fc1 forward of the GPT-1.3B MLP: library NT + HIP bias-GELU pass, own NT + pass, and the own
    NT with bias + GELU + pre-activation in the overlapped epilogue (ops/gemm.mm_nt_bias_gelu)"""
    import os
    from paddle_hackathon_amd.ops import hip
    T, K, N = 32768, 2048, 8192
    x, wt = r(T, K), r(N, K)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    act, pre = G.mm_nt_bias_gelu(x, wt, b)
    ref_pre = x.float() @ wt.float().t()
    ref_act = torch.nn.functional.gelu(ref_pre + b.float(), approximate="tanh")
    e1 = ((pre.float() - ref_pre).abs().max() / ref_pre.abs().max()).item()
    e2 = ((act.float() - ref_act).abs().max() / ref_act.abs().max()).item()
    print(f"fused gelu epilogue: pre rel_err {e1:.2e}  act rel_err {e2:.2e}", flush=True)
    fl = 2.0 * T * K * N

    def lib():
        os.environ["PHA_GEMM_IMPL"] = "library"
        h = G.mm_nt(x, wt)
        os.environ.pop("PHA_GEMM_IMPL")
        return hip.bias_gelu_fwd(h, b, True)

    def own_pass():
        h = G.gemm_p(x, wt, False, False)
        return hip.bias_gelu_fwd(h, b, True)
    res = {"lib+pass": timeit(lib), "own+pass": timeit(own_pass), "own fused": timeit(lambda: G.mm_nt_bias_gelu(x, wt, b)),
           "own gemm only": timeit(lambda: G.gemm_p(x, wt, False, False, bias=b))}
    os.environ.pop("PHA_GEMM_IMPL", None)
    for k, v in res.items():
        print(f"fc1 fwd {k:14s}: {v * 1e6:7.1f} us  {fl / v / 1e12:6.0f} TF  (x24 layers: {v * 24e3:.2f} ms)", flush=True)


def rstage():
    """NT on gemm4p: LDS-DMA staging vs register staging (EPI_RSTAGE) vs hipBLASLt — numerics
    (bitwise equal outputs expected: same MFMA order) and speed at the GPT NT shapes"""
    torch.manual_seed(0)
    for (M, N, K) in [(264, 520, 128), (1032, 2056, 512), (4096, 4096, 1024), (296, 8, 64)]:
        a, b = r(M, K), r(N, K)
        bias = torch.randn(N, device="cuda")
        for bb in (None, bias):
            c0 = G.gemm_p(a, b, False, False, bias=bb)
            c1 = G.gemm_p(a, b, False, False, bias=bb, epi_extra=G.EPI_RSTAGE)
            torch.cuda.synchronize()
            print(f"rstage check M={M} N={N} K={K} bias={bb is not None}: equal={torch.equal(c0, c1)} "
                  f"max_diff={(c0.float() - c1.float()).abs().max().item():.2e}", flush=True)
    a, b = r(4096, 2048), r(8192, 2048)
    bias = torch.randn(8192, device="cuda", dtype=torch.bfloat16)
    pre0 = torch.empty(4096, 8192, device="cuda", dtype=torch.bfloat16)
    pre1 = torch.empty_like(pre0)
    g0 = G.gemm_p(a, b, False, False, bias=bias, gelu_aux=pre0)
    g1 = G.gemm_p(a, b, False, False, bias=bias, gelu_aux=pre1, epi_extra=G.EPI_RSTAGE)
    print(f"rstage gelu: equal={torch.equal(g0, g1) and torch.equal(pre0, pre1)}", flush=True)
    T = 32768
    for name, N, K in [("qkv fwd", 6144, 2048), ("qkv dX", 2048, 6144), ("out", 2048, 2048), ("fc1 fwd", 8192, 2048),
                       ("fc1 dX", 2048, 8192), ("fc2 fwd", 2048, 8192), ("fc2 dX", 8192, 2048)]:
        a, b = r(T, K), r(N, K)
        fl = 2.0 * T * N * K
        t0 = timeit(lambda: G.gemm_p(a, b, False, False))
        t1 = timeit(lambda: G.gemm_p(a, b, False, False, epi_extra=G.EPI_RSTAGE))
        tl = timeit(lambda: a @ b.t())
        print(f"{name:8s} {T}x{N}x{K}: dma {fl / t0 / 1e12:6.0f} TF  rstage {fl / t1 / 1e12:6.0f} TF  "
              f"lib {fl / tl / 1e12:6.0f} TF", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "rstage":
        rstage()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "gelu":
        gelu()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "nnform":
        nnform()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "paths":
        paths()
        sys.exit(0)
    check()
    if len(sys.argv) < 2 or sys.argv[1] != "check":
        bench()
