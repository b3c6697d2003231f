"""Sustained-load weight-gradient (TN: dW = X^T dY, K = 32768 tokens) timing at the GPT-3 1.3B
shapes: own gemm4p (default split policy, and unsplit) vs hipBLASLt (a^T @ b), mean of the last
second of back-to-back runs. python tools/tn_sustain.py"""
import os
import sys

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402
from tools.g4p_sustain import sustain  # noqa: E402

T = 32768
SHAPES = os.environ.get("SHAPES")


def main():
    for name, M, N in (("fc1 dW", 2048, 8192), ("fc2 dW", 8192, 2048), ("qkv dW", 2048, 6144),
                       ("out dW", 2048, 2048)):
        if SHAPES and name not in SHAPES.split(","):
            continue
        a = torch.randn(T, M, device="cuda").bfloat16()
        b = (torch.randn(T, N, device="cuda") * 0.02).bfloat16()
        fl = 2.0 * T * M * N
        sp = G._splits(M, N, T, a.device)
        var = {"own": lambda: G.gemm_p(a, b, True, True, splits=sp),
               "own1": lambda: G.gemm_p(a, b, True, True, splits=1),
               "lib": lambda: a.t() @ b}
        for extra in os.environ.get("TN_VARIANTS", "").split(","):
            if extra:
                bits = int(extra, 0)
                var[f"own+{extra}"] = lambda bits=bits: G.gemm_p(a, b, True, True, splits=sp, epi_extra=bits)
        res = {k: sustain(f) for k, f in var.items()}
        print(f"{name:7s} M={M} N={N} splits={sp}  " +
              "  ".join(f"{k} {t * 1e6:7.1f} us {fl / t / 1e12:6.0f} TF/s" for k, t in res.items()), flush=True)


if __name__ == "__main__":
    main()
