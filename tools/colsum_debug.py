"""Decode what gemm4p's TN column-sum path sums: 1 tile x 1 K-tile with structured B."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from paddle_hackathon_amd.ops import gemm as G

torch.set_printoptions(linewidth=200, precision=1, sci_mode=False)
M, N, K = 256, 256, 64
a = torch.zeros(K, M, dtype=torch.bfloat16, device="cuda")
cases = {"ones": torch.ones(K, N), "col": torch.arange(N).float().expand(K, N) % 64,
         "k": torch.arange(K).float()[:, None].expand(K, N)}
for name, b in cases.items():
    b = b.contiguous().bfloat16().cuda()
    c, part = G.gemm_p(a, b, True, True, colsum=True)
    torch.cuda.synchronize()
    print(name, "expected", b.float().sum(0)[:40].tolist())
    for r in range(part.shape[0]):
        print(" row", r, part[r, :40].tolist())
        print("   cols 128..", part[r, 128:168].tolist())

# weight of each k in the column sums (1 = counted once)
wts = []
for kk in range(K):
    b = torch.zeros(K, N)
    b[kk] = 1.0
    c, part = G.gemm_p(a, b.bfloat16().cuda(), True, True, colsum=True)
    wts.append(part[:, 0].tolist())
print("per-k weights (rows):", wts)
