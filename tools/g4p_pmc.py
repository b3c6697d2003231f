"""PMC driver: the long-K (32768x2048x8192) and short-K (32768x8192x2048) NT products on gemm4p
and on hipBLASLt, a few launches each, for rocprofv3 --pmc passes (per-dispatch counters)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402


def main():
    torch.manual_seed(0)
    for (M, N, K) in ((32768, 2048, 8192), (32768, 8192, 2048)):
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(N, K, device="cuda").bfloat16()
        for sched in ("0", "1"):   # plain / early-release schedule (dispatch order: 3 + 3, then library)
            os.environ["PHA_G4P_EARLY"] = sched
            for _ in range(3):
                G.gemm_p(a, b, False, False)
        for _ in range(3):
            a @ b.t()
        torch.cuda.synchronize()
        del a, b


if __name__ == "__main__":
    main()
