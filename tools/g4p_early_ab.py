"""gemm4p EARLY schedule A/B on the GPT-3 1.3B step's products (every layout the step uses):
bitwise comparison with the default schedule, then interleaved timing (median of 5) of default,
EARLY and hipBLASLt.  python tools/g4p_early_ab.py"""
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402

T = 32768


def t1(fn, iters=8):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


def cases():
    for name, N, K in (("qkv fwd", 6144, 2048), ("out fwd", 2048, 2048), ("fc2 fwd", 2048, 8192),
                       ("qkv dX", 2048, 6144), ("fc1 dX", 2048, 8192), ("fc2 dX", 8192, 2048)):
        x, wt, b = r(T, K), r(N, K), torch.randn(N, device="cuda")
        yield (f"NT {name} {T}x{N}x{K}", 2.0 * T * N * K,
               lambda e, x=x, wt=wt, b=b: G.gemm_p(x, wt, bias=b, epi_extra=e), lambda x=x, wt=wt, b=b: torch.addmm(b.bfloat16(), x, wt.t()))
    x, wt, b = r(T, 2048), r(8192, 2048), torch.randn(8192, device="cuda")
    pre = torch.empty(T, 8192, dtype=torch.bfloat16, device="cuda")
    yield ("NT fc1 fwd +GELU 32768x8192x2048", 2.0 * T * 8192 * 2048,
           lambda e: G.gemm_p(x, wt, bias=b, gelu_aux=pre, epi_extra=e), None)
    for name, M, N in (("qkv dW", 2048, 6144), ("out dW", 2048, 2048), ("fc1 dW", 2048, 8192), ("fc2 dW", 8192, 2048)):
        a, dy = r(T, M), r(T, N)
        sp = G._splits(M, N, T, a.device)
        yield (f"TN {name} {M}x{N}x{T} split{sp}", 2.0 * T * M * N,
               lambda e, a=a, dy=dy, sp=sp: G.gemm_p(a, dy, True, True, splits=sp, epi_extra=e), lambda a=a, dy=dy: a.t() @ dy)
    dl, E = r(T, 50304), r(50304, 2048)
    yield ("NN head dh 32768x2048x50304", 2.0 * T * 2048 * 50304,
           lambda e: G.nn_p(dl, E, epi_extra=e), lambda: dl @ E)


def main():
    import os
    quick = os.environ.get("G4P_QUICK") == "1"   # a subset for variant-library A/Bs
    tot = {"g4p": 0.0, "early": 0.0}
    for case in cases():
        if case is None:
            continue
        if quick and not any(k in case[0] for k in ("fc2 fwd", "fc2 dX", "fc1 dW", "qkv fwd")):
            continue
        name, fl, f, lib = case
        c0 = f(0).clone()
        c1 = f(G.EPI_EARLY)
        eq = torch.equal(c0, c1)
        var = {"g4p": lambda: f(0), "early": lambda: f(G.EPI_EARLY)}
        if lib is not None:
            var["lib"] = lib
        times = {k: [] for k in var}
        for _ in range(5):
            for k, fn in var.items():
                times[k].append(t1(fn))
        med = {k: statistics.median(v) for k, v in times.items()}
        tot["g4p"] += med["g4p"]
        tot["early"] += med["early"]
        print(f"{name}: bitwise_equal={eq}  " + "  ".join(f"{k} {med[k] * 1e6:.0f}us/{fl / med[k] / 1e12:.0f}TF"
                                                        for k in var), flush=True)
    print(f"sum over the listed products: g4p {tot['g4p'] * 1e3:.2f} ms  early {tot['early'] * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
