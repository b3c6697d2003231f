"""Flash-attention backward outputs of two kernel-library builds compared bit for bit (one process
per build: PHA_KERNELS_LIB selects the library at import).
  python tools/fa_lib_compare.py save OUT.pt      (under PHA_KERNELS_LIB=...)
  python tools/fa_lib_compare.py cmp A.pt B.pt"""
import sys

import torch

sys.path.insert(0, ".")


def save(path):
    from paddle_hackathon_amd.ops import hip
    torch.manual_seed(0)
    out = {}
    for causal, S, Sk in ((True, 2048, 2048), (False, 300, 520), (True, 520, 200)):
        B, H, Hk, D = 2, 8, 2, 128
        q = torch.randn(B, S, H, D, device="cuda").bfloat16().requires_grad_(True)
        k = torch.randn(B, Sk, Hk, D, device="cuda").bfloat16().requires_grad_(True)
        v = torch.randn(B, Sk, Hk, D, device="cuda").bfloat16().requires_grad_(True)
        o = hip.FlashAttention.apply(q, k, v, causal, None)
        g = torch.autograd.grad(o, (q, k, v), torch.randn_like(o))
        out[f"{causal}_{S}_{Sk}"] = [t.cpu() for t in (o,) + g]
    torch.save(out, path)


def cmp(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    ok = True
    for key in A:
        for name, x, y in zip(("o", "dq", "dk", "dv"), A[key], B[key]):
            eq = torch.equal(x, y)
            ok &= eq
            print(f"{key} {name}: bitwise_equal={eq} max_diff={(x.float() - y.float()).abs().max().item():.3g}")
    print("ALL EQUAL" if ok else "DIFFERENT")


if __name__ == "__main__":
    save(sys.argv[2]) if sys.argv[1] == "save" else cmp(sys.argv[2], sys.argv[3])
