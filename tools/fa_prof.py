"""Flash-attention backward at the GPT-3 1.3B shape (B=8, S=2048, H=16, D=128, causal) for
rocprofv3: PHA_FA_BWD=fused|v2 picks the path; runs the forward once and the backward N times."""
import os
import sys

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import hip  # noqa: E402


def main(n=int(os.environ.get("FA_ITERS", "5"))):
    B, S, H, D = 8, 2048, 16, 128
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device="cuda").bfloat16().requires_grad_(True) for _ in range(3))
    o = hip.FlashAttention.apply(q, k, v, True, None)
    do = torch.randn_like(o)
    for _ in range(n):
        torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
