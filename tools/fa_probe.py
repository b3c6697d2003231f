"""Step-by-step flash-attention probe (each launch synchronised and reported)."""
import sys
import time

import torch
import torch.nn.functional as TF

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import hip  # noqa: E402


def ref(q, k, v, causal):
    qt, kt, vt = (t.float().transpose(1, 2) for t in (q, k, v))
    return TF.scaled_dot_product_attention(qt, kt, vt, is_causal=causal).transpose(1, 2)


def run(B, S, H, D, causal, bwd):
    torch.manual_seed(0)
    q = torch.randn(B, S, H, D, device="cuda").bfloat16().requires_grad_(bwd)
    k = torch.randn(B, S, H, D, device="cuda").bfloat16().requires_grad_(bwd)
    v = torch.randn(B, S, H, D, device="cuda").bfloat16().requires_grad_(bwd)
    t0 = time.time()
    print(f"fwd B{B} S{S} H{H} D{D} causal={causal} ...", flush=True)
    o = hip.FlashAttention.apply(q, k, v, causal, None)
    torch.cuda.synchronize()
    err = (o.float() - ref(q.detach(), k.detach(), v.detach(), causal)).abs().max().item()
    print(f"  fwd ok {time.time() - t0:.3f}s maxerr={err:.4f}", flush=True)
    if bwd:
        t0 = time.time()
        o.backward(torch.randn_like(o))
        torch.cuda.synchronize()
        print(f"  bwd ok {time.time() - t0:.3f}s", flush=True)


if __name__ == "__main__":
    run(1, 128, 1, 128, False, False)
    run(1, 128, 1, 128, True, False)
    run(2, 200, 3, 64, True, False)
    run(1, 128, 1, 128, False, True)
    run(2, 200, 3, 64, True, True)
    run(8, 2048, 16, 128, True, True)
    print("ALL OK", flush=True)
