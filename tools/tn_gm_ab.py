"""group_m A/B of the own TN weight-gradient products of the GPT-3 1.3B step (gemm4p, split-K as
the static policy picks): group_m 1 / 2 / 4 (default) / 8, interleaved, median of 5, bitwise
cross-check.   python tools/tn_gm_ab.py"""
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


def main():
    for name, M, N in (("qkv dW", 2048, 6144), ("out dW", 2048, 2048), ("fc1 dW", 2048, 8192), ("fc2 dW", 8192, 2048)):
        a = (torch.rand(T, M, device="cuda") * 2 - 1).bfloat16()
        dy = (torch.rand(T, N, device="cuda") * 2 - 1).bfloat16()
        sp = G._splits(M, N, T, a.device)
        fl = 2.0 * T * M * N
        var = {f"gm{g}": (lambda g=g: G.gemm_p(a, dy, True, True, splits=sp, group_m=g, epi_extra=G.EPI_EARLY))
               for g in (1, 2, 4, 8)}
        var["gm4_noearly"] = lambda: G.gemm_p(a, dy, True, True, splits=sp, group_m=4)
        ref = var["gm4"]()
        same = all(torch.equal(f(), ref) for f in var.values())
        ts = {k: [] for k in var}
        for _ in range(5):
            for k, f in var.items():
                f()
                ts[k].append(t1(f))
        print(f"{name} {M}x{N}x{T} split{sp} TF/s: " +
              " ".join(f"{k} {fl / statistics.median(v) / 1e12:6.0f}" for k, v in ts.items()) + f"  bitwise_equal={same}",
              flush=True)


if __name__ == "__main__":
    main()
