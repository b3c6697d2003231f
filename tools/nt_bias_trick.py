"""Library NT products with and without a (zero) bias: the bias-epilogue GEMM is a different
hipBLASLt / TunableOp entry (GemmAndBias) whose solution can be faster for the same shape. Times
a @ bt^T against addmm(0, a, bt^T) for GPT-3 1.3B's dX shapes (M = 32768 tokens), with the in-tree
TunableOp database loaded as bench.py does. python tools/nt_bias_trick.py"""
import sys

import torch

sys.path.insert(0, ".")


def _t(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    from paddle_hackathon_amd.incubate import autotune
    n = autotune.enable_gemm_tuning(tune=False)
    print(f"tunableop entries {n}")
    M = 32768
    torch.manual_seed(0)
    for (N, K, name) in [(2048, 8192, "fc1 dX"), (2048, 2048, "out dX"), (2048, 6144, "qkv dX"),
                         (8192, 2048, "fc2 dX"), (6144, 2048, "qkv fwd"), (2048, 8192, "fc2 fwd")]:
        a = torch.randn(M, K, device="cuda").bfloat16()
        bt = torch.randn(N, K, device="cuda").bfloat16()
        z = torch.zeros(N, device="cuda").bfloat16()
        t0 = _t(lambda: a @ bt.t())
        t1 = _t(lambda: torch.addmm(z, a, bt.t()))
        t0b = _t(lambda: a @ bt.t())
        fl = 2 * M * N * K
        print(f"{name:8s} N={N:5d} K={K:5d}  mm {min(t0, t0b):.4f} ms ({fl / min(t0, t0b) / 1e9:.0f} TF/s)  "
              f"addmm(0) {t1:.4f} ms ({fl / t1 / 1e9:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
