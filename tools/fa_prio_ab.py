"""Wave-priority A/B of the 8-wave flash-attention kernels (PHA_FA_PRIO 0 / 1 / 2, see
csrc/kernels/fa_common.h FaStrides::prio) at the GPT-3 1.3B bench shape (B=16, S=2048, H=16,
D=128, causal), alternated, with a bitwise check against PHA_FA_PRIO=0.

  python tools/fa_prio_ab.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_hackathon_amd.ops import hip  # noqa: E402


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


def main():
    B, S, H, D = 16, 2048, 16, 128
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16).requires_grad_(True) for _ in range(3))
    fl = 4 * B * H * S * S * D / 2
    do = torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16)
    base = {}
    for rep in range(2):
        for prio in ("0", "1", "2"):
            os.environ["PHA_FA_PRIO"] = prio
            with torch.no_grad():
                o = hip.FlashAttention.apply(q, k, v, True, None)
                tf = timeit(lambda: hip.FlashAttention.apply(q, k, v, True, None))
            og = hip.FlashAttention.apply(q, k, v, True, None)
            g = torch.autograd.grad(og, (q, k, v), do, retain_graph=True)
            tb = timeit(lambda: torch.autograd.grad(og, (q, k, v), do, retain_graph=True), 5)
            if prio == "0":
                base = {"o": o, "g": g}
            eq = torch.equal(o, base["o"]) and all(torch.equal(a, b) for a, b in zip(g, base["g"]))
            print(f"rep {rep} prio {prio}: fwd {tf * 1e3:.3f} ms {fl / tf / 1e12:6.1f} TF   "
                  f"bwd {tb * 1e3:.3f} ms {2.5 * fl / tb / 1e12:6.1f} TF   bitwise_eq_prio0={eq}", flush=True)


if __name__ == "__main__":
    main()
