"""LN backward at the GPT-3 1.3B shape ([32768, 2048] bf16, fp32 weights, fused residual
gradient): the prefetching one-wave-per-SIMD sweep (default) vs the two-waves-per-SIMD kernel
(PHA_LN_BWD_PF=0), alternating; equality of their outputs."""
import os
import sys

import torch

sys.path.insert(0, ".")


def main():
    from paddle_hackathon_amd.ops import hip
    R, H = 32768, 2048
    torch.manual_seed(0)
    x = torch.randn(R, H, device="cuda").bfloat16()
    dy, dres = torch.randn_like(x), torch.randn_like(x)
    w = torch.rand(H, device="cuda") + 0.5
    b = torch.randn(H, device="cuda")
    y, mean, rstd = hip.layer_norm_fwd(x, w, b, 1e-5)
    outs = {}
    for rnd in range(2):
        for pf in ("1", "0"):
            os.environ["PHA_LN_BWD_PF"] = pf
            f = lambda: hip.layer_norm_bwd(dy, x, w, mean, rstd, True, dres=dres)
            outs[pf] = f()
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
            print(f"pf={pf} {t * 1e3:7.1f} us/call  {4 * R * H * 2 / t / 1e9:.2f} TB/s", flush=True)
    os.environ.pop("PHA_LN_BWD_PF")
    a, b2 = outs["1"], outs["0"]
    print("dx equal:", torch.equal(a[0], b2[0]), " dw max rel:", ((a[1] - b2[1]).abs().max() / b2[1].abs().max()).item(),
          " db max rel:", ((a[2] - b2[2]).abs().max() / b2[2].abs().max()).item())


if __name__ == "__main__":
    main()
