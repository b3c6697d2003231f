"""Flash attention at the BERT-base shape (B=32, S=512, H=12, D=64, packed QKV, non-causal): forward
and forward+backward time of the own kernels without / with the key-padding mask and dropout,
next to torch SDPA on the same device, with the achieved TF/s (2 GEMMs forward, 5 backward)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from paddle_hackathon_amd.ops import hip as H


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


B, S, Hn, D = 32, 512, 12, 64
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(B, S, Hn, 3 * D, device="cuda", generator=g).bfloat16().requires_grad_(True)
mask = torch.zeros(B, 1, 1, S, device="cuda")
mask[:, :, :, S - 37:] = -1e4
fl_f = 4.0 * B * Hn * S * S * D
for name, m, p in (("plain", None, 0.0), ("mask", mask, 0.0), ("dropout", None, 0.1), ("mask+dropout", mask, 0.1)):
    def fwd():
        return H.flash_attention_packed_ext(qkv, False, None, m, p)
    o = fwd()
    if o is None:
        print(f"{name:13s} not supported by the ext kernels")
        continue
    do = torch.randn_like(o)
    tf = timeit(lambda: fwd())

    def fb():
        o = fwd()
        torch.autograd.grad(o, qkv, do)
    tfb = timeit(fb)
    print(f"{name:13s} fwd {tf * 1e3:7.1f} us ({fl_f / tf / 1e9:6.1f} TF/s)   fwd+bwd {tfb * 1e3:7.1f} us "
          f"({3.5 * fl_f / tfb / 1e9:6.1f} TF/s)", flush=True)
q, k, v = (qkv[..., i * D:(i + 1) * D].transpose(1, 2).contiguous().detach().requires_grad_(True) for i in range(3))
for name, m, p in (("sdpa plain", None, 0.0), ("sdpa mask+drop", mask, 0.1)):
    def fwd():
        return torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=None if m is None else m.bfloat16(),
                                                                dropout_p=p)
    o = fwd()
    do = torch.randn_like(o)
    tf = timeit(lambda: fwd())

    def fb():
        o = fwd()
        torch.autograd.grad(o, (q, k, v), do)
    tfb = timeit(fb)
    print(f"{name:13s} fwd {tf * 1e3:7.1f} us ({fl_f / tf / 1e9:6.1f} TF/s)   fwd+bwd {tfb * 1e3:7.1f} us "
          f"({3.5 * fl_f / tfb / 1e9:6.1f} TF/s)", flush=True)
