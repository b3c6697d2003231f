"""LayerNorm forward / backward at the GPT-3 1.3B shape (32768 x 2048 bf16, fp32 weights) and
BERT (16384 x 768): time per call and effective HBM bandwidth."""
import sys
import time
import torch
sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import hip  # noqa: E402


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


for R, H in ((32768, 2048), (16384, 768)):
    x = torch.randn(R, H, device="cuda").bfloat16()
    r = torch.randn(R, H, device="cuda").bfloat16()
    w = torch.rand(H, device="cuda") + 0.5
    b = torch.randn(H, device="cuda")
    y, mean, rstd, hs = hip.layer_norm_fwd(x, w, b, 1e-5, residual=r)
    dy = torch.randn_like(y)
    fwd = t(lambda: hip.layer_norm_fwd(x, w, b, 1e-5, residual=r))
    bwd = t(lambda: hip.layer_norm_bwd(dy, hs, w, mean, rstd, True, dres=dy))
    nb = R * H * 2
    print(f"{R}x{H}: add+LN fwd {fwd:.1f} us ({4 * nb / fwd / 1e6:.2f} TB/s)   LN bwd+dres {bwd:.1f} us "
          f"({4 * nb / bwd / 1e6:.2f} TB/s)")
