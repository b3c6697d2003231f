"""Weight-gradient GEMM with and without the column-sum (bias gradient) path: the GPT-3 1.3B
micro-batch-48 dW shapes, plain TN + the old col_sum pass vs TN with G4P_COLSUM (+ finish)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from paddle_hackathon_amd.ops import gemm as G
from paddle_hackathon_amd.ops import hip as H

T = 98304
SHAPES = [("qkv dW", 2048, 6144), ("out dW", 2048, 2048), ("fc1 dW", 2048, 8192), ("fc2 dW", 8192, 2048)]


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


g = torch.Generator(device="cuda").manual_seed(0)
tot = [0.0, 0.0, 0.0]
for name, M, N in SHAPES:
    x = (torch.rand(T, M, device="cuda", generator=g) - 0.5).bfloat16()
    dy = (torch.rand(T, N, device="cuda", generator=g) - 0.5).bfloat16()
    sp = G._splits(M, N, T, x.device)
    t_tn = timeit(lambda: G.gemm_p(x, dy, True, True, splits=sp))
    t_cs = timeit(lambda: H.col_sum(dy))
    t_new = timeit(lambda: G.mm_tn_db(x, dy))
    tot[0] += t_tn
    tot[1] += t_cs
    tot[2] += t_new
    print(f"{name:7s} {M}x{N}x{T} split {sp}: TN {t_tn:8.1f} us + col_sum {t_cs:6.1f} = {t_tn + t_cs:8.1f} | "
          f"TN+colsum {t_new:8.1f} us  ({(t_new / (t_tn + t_cs) - 1) * 100:+.1f} %)", flush=True)
print(f"per layer: old {tot[0] + tot[1]:.1f} us, new {tot[2]:.1f} us; per step x24: {24 * (tot[2] - tot[0] - tot[1]) / 1e3:+.2f} ms")
