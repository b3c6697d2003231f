"""Flash attention at the GPT-3 1.3B step shape (B=16, S=2048, H=16, D=128): our forward and
backward against torch's SDPA (the ROCm flash backend), causal and not, in TF/s (causal FLOPs
halved). Env FA_B / FA_S override the batch / sequence."""
import os
import sys
import time

import torch
import torch.nn.functional as TF

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import hip  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters)
    return best


def main():
    B, S, H, D = int(os.environ.get("FA_B", 16)), int(os.environ.get("FA_S", 2048)), 16, 128
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16).requires_grad_(True) for _ in range(3))
    for causal in (True, False):
        fl = 4 * B * H * S * S * D / (2 if causal else 1)
        with torch.no_grad():
            tf = timeit(lambda: hip.FlashAttention.apply(q, k, v, causal, None))
        o = hip.FlashAttention.apply(q, k, v, causal, None)
        do = torch.randn_like(o)
        tb = timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True), 5)
        qt, kt, vt = (x.detach().transpose(1, 2).requires_grad_(True) for x in (q, k, v))
        with torch.no_grad():
            sf = timeit(lambda: TF.scaled_dot_product_attention(qt, kt, vt, is_causal=causal))
        os_ = TF.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
        dos = do.transpose(1, 2)
        sb = timeit(lambda: torch.autograd.grad(os_, (qt, kt, vt), dos, retain_graph=True), 5)
        print(f"causal={causal}: ours fwd {tf * 1e3:.3f} ms {fl / tf / 1e12:.0f} TF  bwd {tb * 1e3:.3f} ms "
              f"{2.5 * fl / tb / 1e12:.0f} TF | sdpa fwd {sf * 1e3:.3f} ms {fl / sf / 1e12:.0f} TF  bwd "
              f"{sb * 1e3:.3f} ms {2.5 * fl / sb / 1e12:.0f} TF", flush=True)


if __name__ == "__main__":
    main()
