"""Flash-attention backward A/B at the GPT-3 1.3B step shape (B=16, S=2048, H=16, D=128, causal):
dK/dV kernel v3 (pipelined, default) vs v2 (PHA_FA_DKDV=v2), plus the forward. Gradients of the
two paths are compared with each other and with an fp32 reference on a smaller batch."""
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
    B, S, H, D = int(os.environ.get("FA_B", 16)), 2048, 16, 128
    causal = os.environ.get("FA_CAUSAL", "1") == "1"
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16).requires_grad_(True) for _ in range(3))
    fl = 4 * B * H * S * S * D / (2 if causal else 1)
    quick = os.environ.get("FA_QUICK") == "1"   # v3 paths only (variant-library A/B runs)
    outs = {}
    for name in (("v3",) if quick else ("v2", "v3")):
        os.environ["PHA_FA_FWD"] = name
        with torch.no_grad():
            outs[name] = hip.FlashAttention.apply(q, k, v, causal, None)
            t = timeit(lambda: hip.FlashAttention.apply(q, k, v, causal, None))
        print(f"fwd {name}: {t * 1e3:.3f} ms  {fl / t / 1e12:.1f} TF", flush=True)
    if not quick:
        print(f"  fwd v3 vs v2 max diff {(outs['v2'].float() - outs['v3'].float()).abs().max().item():.5f}", flush=True)
    o = hip.FlashAttention.apply(q, k, v, causal, None)
    do = torch.randn_like(o)
    grads = {}
    for name, env, dqe in ((("v3", "v3", "v3"),) if quick else (("v2", "v2", "v2"), ("v3dkdv", "v3", "v2"), ("v3", "v3", "v3"))):
        os.environ["PHA_FA_DKDV"] = env
        os.environ["PHA_FA_DQ"] = dqe
        grads[name] = torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
        t = timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True), 5)
        print(f"bwd {name}: {t * 1e3:.3f} ms  {2.5 * fl / t / 1e12:.1f} TF (useful flops)", flush=True)
    if quick:
        return
    for n, a, b in zip("qkv", grads["v2"], grads["v3"]):
        print(f"  d{n} v3 vs v2 max diff {(a.float() - b.float()).abs().max().item():.5f} "
              f"(scale {a.float().abs().max().item():.3f})", flush=True)
    # fp32 reference on 2 sequences
    qr, kr, vr = (x[:2].detach().float().transpose(1, 2).requires_grad_(True) for x in (q, k, v))
    orf = TF.scaled_dot_product_attention(qr, kr, vr, is_causal=causal)
    gref = torch.autograd.grad(orf, (qr, kr, vr), do[:2].float().transpose(1, 2))
    for n, a, r in zip("qkv", grads["v3"], gref):
        r = r.transpose(1, 2)
        print(f"  v3 d{n} max err vs fp32 {(a[:2].float() - r).abs().max().item():.4f} (scale {r.abs().max().item():.3f})",
              flush=True)


if __name__ == "__main__":
    main()
