"""PMC driver: one NT product (default the long-K 32768x2048x8192) on gemm8w, gemm8w with the
second wave half at setprio 1, gemm4p and hipBLASLt, 3 launches each (dispatch order), for
rocprofv3 --pmc passes.  python tools/g8w_pmc.py [M N K]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (32768, 2048, 8192)
    torch.manual_seed(0)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    for fn in (lambda: G.gemm_8w(a, b), lambda: G.gemm_8w(a, b, epi_extra=2), lambda: G.gemm_p(a, b),
               lambda: a @ b.t()):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
