"""gemm4w NT / NN / TN / TT at 32768 x 8192 x 2048 (fc1 shape, bf16 random), two launches each,
for rocprofv3 PMC passes (the layouts are distinct kernel instantiations)."""
import sys
import torch
sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402
M, N, K = 32768, 8192, 2048
r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
a, at = r(M, K), r(K, M)
b, bt = r(K, N), r(N, K)
for _ in range(2):
    G.gemm(a, bt, False, False)
    G.gemm(a, b, False, True)
    G.gemm(at, bt, True, False)
    G.gemm(at, b, True, True)
torch.cuda.synchronize()
print("done")
