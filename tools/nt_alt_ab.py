"""The long-K NT products of the GPT-3 1.3B step (N = 2048, K = 6144 / 8192) on the own kernel in
alternative forms vs hipBLASLt: NT (x @ W^T with the cached transposed weight) with group_m 1..16,
and the NN form (x @ W on the [K, N] weight, gemm4p's transposed-store layout). Interleaved,
median of 5, bitwise cross-checks.   python tools/nt_alt_ab.py"""
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


def main():
    for name, N, K in (("fc2 fwd", 2048, 8192), ("fc1 dX", 2048, 8192), ("qkv dX", 2048, 6144),
                       ("out fwd", 2048, 2048), ("qkv fwd", 6144, 2048)):
        x, w = r(T, K), r(K, N)
        wt = w.t().contiguous()
        fl = 2.0 * T * N * K
        variants = {"lib": lambda: x @ w}
        for gm in (1, 2, 4, 8, 16):
            variants[f"nt_gm{gm}"] = (lambda gm=gm: G.gemm_p(x, wt, group_m=gm, epi_extra=G.EPI_EARLY))
        variants["nn"] = lambda: G.nn_p(x, w)
        ref = variants["nt_gm4"]().float()
        errs = {k: (f().float() - ref).abs().max().item() for k, f in variants.items() if k != "lib"}
        times = {k: [] for k in variants}
        for _ in range(5):
            for k, f in variants.items():
                f()
                times[k].append(t1(f))
        line = " ".join(f"{k} {fl / statistics.median(v) / 1e12:6.0f}" for k, v in times.items())
        print(f"{name} {T}x{N}x{K} TF/s: {line}   max|diff| vs nt_gm4: {max(errs.values()):.3g}", flush=True)


if __name__ == "__main__":
    main()
