"""gemm4p tile-walk panel height (group_m) for the GPT-3 1.3B weight gradients (TN, K = 98,304
tokens at micro-batch 48), through ops.gemm.mm_tn as the model calls it (split-K picks included):
python tools/g4p_groupm_tn_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402


def _t(fn, it=8):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


K = 98304
for name, M, N in [("qkv dW", 2048, 6144), ("out dW", 2048, 2048), ("fc1 dW", 2048, 8192), ("fc2 dW", 8192, 2048)]:
    x = (torch.randn(K, M, device="cuda") * 0.1).bfloat16()
    dy = (torch.randn(K, N, device="cuda") * 0.1).bfloat16()
    row = [f"{name} {M}x{N}x{K}:"]
    for gm in (1, 2, 4, 8, 16):
        os.environ["PHA_G4P_GROUP_M"] = str(gm)
        us = _t(lambda: G.mm_tn(x, dy))
        row.append(f"gm{gm} {us:7.1f} us ({2.0 * M * N * K / us / 1e6:5.0f} TF/s)")
    print("  ".join(row), flush=True)
    del x, dy
