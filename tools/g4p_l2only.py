"""Is gemm4p's long-K NT main loop latency-bound on HBM / MALL? The same schedule with every DMA
re-reading the tile's first K-tile (EPI_L2ONLY: L2-resident operands, timing only) against the
normal run and hipBLASLt, sustained load. python tools/g4p_l2only.py"""
import sys

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402
sys.path.insert(0, "tools")
from g4p_sustain import sustain  # noqa: E402

T = 32768


def main():
    for name, N, K in (("fc2 fwd", 2048, 8192), ("qkv fwd", 6144, 2048)):
        x = torch.randn(T, K, device="cuda").bfloat16()
        wt = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        fl = 2.0 * T * N * K
        var = {"lv8": lambda: G.gemm_p(x, wt, epi_extra=G.EPI_EARLY | (8 << 17)),
               "lv8_l2only": lambda: G.gemm_p(x, wt, epi_extra=G.EPI_EARLY | (8 << 17) | (1 << 21)),
               "lib": lambda: x @ wt.t()}
        res = {k: min(sustain(f) for _ in range(2)) for k, f in var.items()}
        print(f"NT {name} {T}x{N}x{K}: " + "  ".join(f"{k} {v * 1e6:.0f}us/{fl / v / 1e12:.0f}TF" for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
