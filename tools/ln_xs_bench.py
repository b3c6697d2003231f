"""LN backward at the GPT-3 1.3B shape ([32768, 2048] bf16, fp32 weights, fused residual
gradient) with and without the dx column sums (dx_colsum): per-call time of each."""
import sys

import torch

sys.path.insert(0, ".")


def main():
    from paddle_hackathon_amd.ops import hip
    R, H = 32768, 2048
    x = torch.randn(R, H, device="cuda").bfloat16()
    dy, dres = torch.randn_like(x), torch.randn_like(x)
    w = torch.rand(H, device="cuda") + 0.5
    b = torch.randn(H, device="cuda")
    y, mean, rstd = hip.layer_norm_fwd(x, w, b, 1e-5)
    for name, kw in [("plain", {}), ("dx_colsum", {"dx_colsum": torch.bfloat16}), ("plain", {}),
                     ("dx_colsum", {"dx_colsum": torch.bfloat16})]:
        f = lambda: hip.layer_norm_bwd(dy, x, w, mean, rstd, True, dres=dres, **kw)
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            f()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / 50
        print(f"{name:10s} {t * 1e3:7.1f} us/call  {4 * R * H * 2 / t / 1e9:.2f} TB/s (dy, x, dres, dx)", flush=True)


if __name__ == "__main__":
    main()
