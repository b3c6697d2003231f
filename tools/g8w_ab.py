"""gemm8w (8 waves, two per SIMD) vs gemm4p (EARLY) vs hipBLASLt on the GPT-3 1.3B NT products:
numerics vs an fp32 reference on a slice, then interleaved timing (median of 5 rounds).
python tools/g8w_ab.py [quick]"""
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402

T = 32768


def t1(fn, iters=6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


def check():
    for (M, N, K) in ((256, 256, 64), (512, 768, 192), (1000, 2048 + 8, 640), (4096, 2048, 8192), (264, 136, 128)):
        a, bt, b = r(M, K), r(N, K), torch.randn(N, device="cuda")
        ref = a.float() @ bt.float().t() + b
        got = G.gemm_8w(a, bt, bias=b).float()
        err = ((got - ref).abs() / (ref.abs() + 1.0)).max().item()
        got0 = G.gemm_8w(a, bt).float()
        err0 = ((got0 - (ref - b)).abs() / (ref.abs() + 1.0)).max().item()
        print(f"check {M}x{N}x{K}: max rel err bias {err:.3e} plain {err0:.3e}", flush=True)
        assert err < 2e-2 and err0 < 2e-2


def main():
    check()
    quick = len(sys.argv) > 1
    shapes = (("qkv fwd", 6144, 2048), ("out fwd", 2048, 2048), ("fc2 fwd", 2048, 8192), ("qkv dX", 2048, 6144),
              ("fc1 dX", 2048, 8192), ("fc2 dX", 8192, 2048), ("fc1 fwd", 8192, 2048), ("head", 50304, 2048))
    tot = {}
    for name, N, K in shapes:
        if quick and name not in ("fc2 fwd", "qkv fwd", "fc2 dX"):
            continue
        x, wt, b = r(T, K), r(N, K), torch.randn(N, device="cuda")
        fl = 2.0 * T * N * K
        var = {f"r{rg}{'p' if pr else ''}": (lambda rg=rg, pr=pr: G.gemm_8w(x, wt, bias=b, epi_extra=(rg << 8) | pr))
               for rg in (2, 3, 6) for pr in (0, 2)}
        var.update({"g4p": lambda: G.gemm_p(x, wt, bias=b), "lib": lambda: torch.addmm(b.bfloat16(), x, wt.t())})
        eq = torch.equal(var["r3"](), var["g4p"]()) and torch.equal(var["r2p"](), var["r6"]())
        times = {k: [] for k in var}
        for _ in range(5):
            for k, fn in var.items():
                times[k].append(t1(fn))
        med = {k: statistics.median(v) for k, v in times.items()}
        for k in med:
            tot[k] = tot.get(k, 0.0) + med[k]
        print(f"NT {name} {T}x{N}x{K}: eq_g4p={eq} " + "  ".join(f"{k} {med[k] * 1e6:.0f}us/{fl / med[k] / 1e12:.0f}TF"
                                                                 for k in var), flush=True)
    print("sum: " + "  ".join(f"{k} {v * 1e3:.2f} ms" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
