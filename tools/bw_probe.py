"""HBM ceilings for the step's streaming kernels: torch fill (write only), sum (read only), copy
(read + write), and a 3-read-1-write add chain at 512 MiB per tensor — the references the LN /
bias-GELU / BN kernels' TB/s are compared against. python tools/bw_probe.py"""
import torch


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it / 1e3


def main():
    n = 256 << 20   # bf16 elements: 512 MiB
    a = torch.randn(n, device="cuda").bfloat16()
    b, c, d = torch.empty_like(a), torch.randn_like(a), torch.randn_like(a)
    B = 2 * n
    for name, fn, byt in (("fill (W)", lambda: b.fill_(1.0), B), ("sum (R)", lambda: a.sum(dtype=torch.float32), B),
                          ("copy (R+W)", lambda: b.copy_(a), 2 * B),
                          ("a+c+d -> b (3R+W)", lambda: torch.add(torch.add(a, c, out=b), d, out=b), 5 * B)):
        s = t(fn)
        print(f"{name:20s} {s * 1e6:8.1f} us  {byt / s / 1e12:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
