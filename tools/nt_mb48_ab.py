"""The GPT-3 1.3B NT products at the bench's micro-batch 48 (M = 98,304 tokens): the own persistent
gemm4p kernel against hipBLASLt (torch @, as the default policy runs them), per shape and summed
over a step (24 layers + head). python tools/nt_mb48_ab.py [tokens]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402


def _t(fn, it=10):
    for _ in range(3):
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
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 48 * 2048
    torch.manual_seed(0)
    tot_own = tot_lib = 0.0
    # (name, N, K, per-step count): forward x W^T on the cached W^T and dX = dY W (both NT here)
    shapes = [("qkv fwd", 6144, 2048, 24), ("out fwd", 2048, 2048, 24), ("fc2 fwd", 2048, 8192, 24),
              ("qkv dX", 2048, 6144, 24), ("out dX", 2048, 2048, 24), ("fc1 dX", 2048, 8192, 24),
              ("fc2 dX", 8192, 2048, 24), ("head logits", 50304, 2048, 1)]
    for name, N, K, cnt in shapes:
        a = (torch.randn(M, K, device="cuda") * 0.1).bfloat16()
        bt = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
        ref = a @ bt.t()
        own = G.gemm_p(a, bt, False, False)
        err = (own.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
        assert err < 2e-2, (name, err)
        tl = _t(lambda: a @ bt.t())
        to = _t(lambda: G.gemm_p(a, bt, False, False))
        fl = 2.0 * M * N * K
        tot_own += to * cnt
        tot_lib += tl * cnt
        print(f"{name:11s} {M}x{N}x{K}: own {to * 1e3:8.1f} us ({fl / to / 1e9:5.0f} TF/s)  "
              f"lib {tl * 1e3:8.1f} us ({fl / tl / 1e9:5.0f} TF/s)  own/lib {to / tl:5.3f}", flush=True)
        del a, bt, ref, own
    print(f"per step (24 layers + head): own {tot_own:.1f} ms  lib {tot_lib:.1f} ms  "
          f"(+{tot_own - tot_lib:.1f} ms on the own kernel)")


if __name__ == "__main__":
    main()
