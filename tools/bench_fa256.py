"""Head dim 256 attention: own generic kernels vs torch SDPA (AOTriton / CK), fwd and fwd+bwd,
B=4 S=2048 H=16 causal bf16."""
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd import ops  # noqa: E402


def t(fn, it=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it * 1e3


for D in (128, 256):
    B, S, H = 4, 2048, 16
    q, k, v = (torch.randn(B, S, H, D, device="cuda").bfloat16().requires_grad_() for _ in range(3))
    do = torch.randn(B, S, H, D, device="cuda").bfloat16()
    own_f = t(lambda: ops.flash_attention(q, k, v, causal=True))
    own_b = t(lambda: torch.autograd.grad(ops.flash_attention(q, k, v, causal=True), (q, k, v), do))
    qt, kt, vt = (x.detach().transpose(1, 2).contiguous().requires_grad_() for x in (q, k, v))
    sd_f = t(lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=True))
    dot = do.transpose(1, 2).contiguous()
    sd_b = t(lambda: torch.autograd.grad(torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=True),
                                         (qt, kt, vt), dot))
    fl = 4.0 * B * H * S * S * D / 2
    print(f"D={D}: own fwd {own_f:.2f} ms ({fl / own_f / 1e9:.0f} TF)  fwd+bwd {own_b:.2f} ms | "
          f"SDPA fwd {sd_f:.2f} ms ({fl / sd_f / 1e9:.0f} TF)  fwd+bwd {sd_b:.2f} ms", flush=True)
