"""gemm4w at 32768 x 8192 x 2048 (fc1 shape, bf16 random), two launches each of the layouts the
framework uses: NT (dX), NN as the transposed store (forward), TN (weight gradient), plus the
library NT for comparison — for rocprofv3 PMC passes (each is its own kernel instantiation)."""
import sys
import torch
sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402
M, N, K = 32768, 8192, 2048
r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
a, at = r(M, K), r(K, M)
b, bt = r(K, N), r(N, K)
for _ in range(2):
    G.gemm(a, bt, False, False)      # NT
    G.nn(a, b)                       # NN via the transposed store
    G.gemm(at, b, True, True)        # TN
    a @ bt.t()                       # library NT
torch.cuda.synchronize()
print("done")
