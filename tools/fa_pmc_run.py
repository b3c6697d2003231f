"""Flash-attention kernels for a PMC pass (tools/gpu_r6_fapmc.sh): the GPT-3 1.3B shape (B=16 S=2048
H=16 D=128 causal: fa_fwd_v3, dK/dV v3, dQ v3) and the BERT-base shape (B=32 S=512 H=12 D=64 with
dropout 0.1 on the packed entry: fa64_fwd / fa64_dkdv / fa64_dq), 3 forward + backward each."""
import sys

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import hip  # noqa: E402

torch.manual_seed(0)
q, k, v = (torch.randn(16, 2048, 16, 128, device="cuda").bfloat16().requires_grad_() for _ in range(3))
for _ in range(3):
    o = hip.flash_attention_any(q, k, v, True, None)
    torch.autograd.grad(o, (q, k, v), torch.ones_like(o))
qkv = torch.randn(32, 512, 12, 192, device="cuda").bfloat16().requires_grad_()
for _ in range(3):
    o = hip.flash_attention_packed_ext(qkv, False, None, None, 0.1)
    torch.autograd.grad(o, qkv, torch.ones_like(o))
torch.cuda.synchronize()
print("ok")
