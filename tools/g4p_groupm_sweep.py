"""gemm4p NT tile-walk panel height (group_m) at the bench's M = 98,304 for the GPT-3 1.3B NT shapes:
python tools/g4p_groupm_sweep.py"""
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
    return s.elapsed_time(e) / it * 1e3


M = 98304
for N, K in [(2048, 2048), (2048, 8192), (6144, 2048)]:
    a = (torch.randn(M, K, device="cuda") * 0.1).bfloat16()
    bt = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    lib = _t(lambda: a @ bt.t())
    row = [f"{M}x{N}x{K}: lib {lib:7.1f} us"]
    for gm in (1, 2, 4, 8, 16, 32):
        us = _t(lambda: G.gemm_p(a, bt, False, False, group_m=gm))
        row.append(f"gm{gm} {us:7.1f}")
    print("  ".join(row), flush=True)
