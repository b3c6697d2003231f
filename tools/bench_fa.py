"""Flash-attention micro-benchmark at the GPT-3 1.3B shape (B=8, S=2048, H=16, D=128, causal):
our forward v1 (4-wave) vs v2 (8-wave, tr-read V) vs torch SDPA, and the backward."""
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
    B, S, H, D = 8, 2048, 16, 128
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16) for _ in range(3))
    causal = True
    fl = 4 * B * H * S * S * D / (2 if causal else 1)
    ref = TF.scaled_dot_product_attention(q.transpose(1, 2).float(), k.transpose(1, 2).float(),
                                          v.transpose(1, 2).float(), is_causal=causal).transpose(1, 2)
    for name, env in (("v1", "1"), ("v2", "0")) if os.environ.get("PHA_FA_BENCH_FAST") != "1" else (("v2", "0"),):
        os.environ["PHA_FA_FWD_V1"] = env
        with torch.no_grad():
            o = hip.FlashAttention.apply(q, k, v, causal, None)
            err = (o.float() - ref).abs().max().item()
            t = timeit(lambda: hip.FlashAttention.apply(q, k, v, causal, None))
        print(f"fwd {name}: {t * 1e3:.3f} ms  {fl / t / 1e12:.1f} TF  max_err {err:.4f}", flush=True)
    qt, kt, vt = (x.transpose(1, 2) for x in (q, k, v))
    t = timeit(lambda: TF.scaled_dot_product_attention(qt, kt, vt, is_causal=causal))
    print(f"fwd torch sdpa: {t * 1e3:.3f} ms  {fl / t / 1e12:.1f} TF", flush=True)
    os.environ["PHA_FA_FWD_V1"] = "0"
    qg, kg, vg = (x.clone().requires_grad_(True) for x in (q, k, v))
    o = hip.FlashAttention.apply(qg, kg, vg, causal, None)
    do = torch.randn_like(o)
    grads = {}
    fast = os.environ.get("PHA_FA_BENCH_FAST") == "1"
    for name, v1, mode in ((("v1", "1", "v2"),) if not fast else ()) + (("v2", "0", "v2"), ("fused", "0", "fused")):
        os.environ["PHA_FA_BWD_V1"] = v1
        os.environ["PHA_FA_BWD"] = mode
        grads[name] = torch.autograd.grad(o, (qg, kg, vg), do, retain_graph=True)
        t = timeit(lambda: torch.autograd.grad(o, (qg, kg, vg), do, retain_graph=True), 5)
        print(f"bwd {name}: {t * 1e3:.3f} ms  {2.5 * fl / t / 1e12:.1f} TF", flush=True)
    # fp32 reference gradients
    qr, kr, vr = (x.detach().transpose(1, 2).float().requires_grad_(True) for x in (q, k, v))
    orf = TF.scaled_dot_product_attention(qr, kr, vr, is_causal=causal)
    gref = torch.autograd.grad(orf, (qr, kr, vr), do.transpose(1, 2).float())
    gref = [x.transpose(1, 2) for x in gref]
    for name in ("v2", "fused"):
        for n, a, r in zip("qkv", grads[name], gref):
            print(f"  {name} d{n} max err vs fp32 {(a.float() - r).abs().max().item():.4f} "
                  f"(scale {r.abs().max().item():.3f})", flush=True)
    qs, ks, vs = (x.transpose(1, 2).clone().requires_grad_(True) for x in (q, k, v))
    os_ = TF.scaled_dot_product_attention(qs, ks, vs, is_causal=causal)
    dos = do.transpose(1, 2)
    t = timeit(lambda: torch.autograd.grad(os_, (qs, ks, vs), dos, retain_graph=True), 5)
    print(f"bwd torch sdpa: {t * 1e3:.3f} ms  {2.5 * fl / t / 1e12:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
